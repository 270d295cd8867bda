"""Drop-in signatures of src/contrastor/utils.py (clustering for ProtoNCE).

``extract_all_emb`` keeps the reference behaviour (src/contrastor/utils.py:11-25:
anchor then positive embedding blocks per batch).  The faiss k-means and the
fastcluster Ward linkage (utils.py:50-160) are the "next" row of SURVEY.md 8f
(they would reuse the scan kernel with an L2 metric, k=1) and raise for now.
"""
import numpy as np
import torch


def extract_all_emb(loader, model, device):
    emb_lst = []
    print("[Runner] - Extracting sentence embedding vectors")
    with torch.no_grad():
        for _, anchor_sample, positive_sample in loader:
            a, p = model.bert_extract(anchor_sample, positive_sample, device)
            emb_lst.append(model.seq2vec(a).cpu().numpy())
            emb_lst.append(model.seq2vec(p).cpu().numpy())
    return np.vstack(emb_lst)


def run_kmeans(proto_nce_config, loader, model, device):
    raise NotImplementedError("k-means for ProtoNCE: SURVEY.md 8f row 3")


def run_hierarchical_clustering(proto_nce_config, loader, model, device):
    raise NotImplementedError("hierarchical clustering for HProtoNCE: SURVEY.md 8f row 3")
