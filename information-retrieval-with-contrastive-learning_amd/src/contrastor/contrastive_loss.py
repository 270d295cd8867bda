"""Drop-in for src/contrastor/contrastive_loss.py (NCELoss).

``NCELoss._compute_info_loss`` keeps the reference semantics exactly (in-batch
NT-Xent over [q; k] with the diagonal removed, optional MoCo queue logits reused
for the k-rows, CE(sum)/2; contrastive_loss.py:56-93) and runs on the irc HIP
kernels (irc_amd/nce.py).  ``_compute_proto_loss`` (ProtoNCE/HProtoNCE,
contrastive_loss.py:95-135) runs on irc_amd.cluster.proto_loss (same negative
prototype draw, exact-fp32 logits, prototype CE kernel).
"""
import random

import torch

from irc_amd.cluster import proto_loss
from irc_amd.nce import info_nce

random.seed(1126)  # module-level seed, as in the reference (contrastive_loss.py:4)


class NCELoss(torch.nn.Module):
    def __init__(self, loss_config):
        super().__init__()
        self.T = loss_config["temperature"]
        if "cluster" in loss_config:
            self.num_cluster = loss_config["cluster"]["num_cluster"]
            self.num_neg_proto = loss_config["cluster"]["num_neg_proto"]

    def _compute_info_loss(self, q, k, queue=None):
        return info_nce(q, k, queue, self.T)

    def _compute_proto_loss(self, q, cluster_result, index):
        return proto_loss(q, cluster_result, index, self.num_cluster, self.num_neg_proto)

    def forward(self, q, k, queue, cluster_result=None, index=None):
        loss = self._compute_info_loss(q, k, queue)
        if cluster_result is not None:
            loss = loss + self._compute_proto_loss(q, cluster_result, index)
        return loss
