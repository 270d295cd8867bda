"""The frozen encoder's split form (irc_amd.bert.BertModel._encode_split): a batch whose
B L rows sit just above a multiple of 32768 (whole waves of every BERT GEMM) runs as
the whole-wave chunk of sequences plus the rest on a side stream.  Every op is per row
except the attention, which is per sequence, so each chunk must equal encoding its
sequences alone bit for bit, and the whole batch agrees with the one-launch form within
the fp32 reassociation of the GEMM kernel choice (reference: the frozen BertModel of
src/contrastor/contrastive_module.py:36-41)."""
import dataclasses

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("B,L", [(512, 65), (512, 68), (600, 56)])
def test_split_encode(gpu, B, L):
    from irc_amd.bert import BERT_BASE, BertModel

    cfg = dataclasses.replace(BERT_BASE, num_hidden_layers=2)
    m = BertModel(cfg, seed=4).to(gpu)
    n1 = m._split_point(B, L)
    assert 0 < n1 < B and n1 * L <= 32768
    g = torch.Generator().manual_seed(B + L)
    ids = torch.randint(1, cfg.vocab_size, (B, L), generator=g)
    lens = torch.randint(8, L + 1, (B,), generator=g)
    lens[0] = L
    mask = (torch.arange(L)[None, :] < lens[:, None]).to(torch.int64)
    ids[mask == 0] = 0
    ids, mask = ids.to(gpu), mask.to(gpu)
    y = m.encode(ids, mask)
    y2 = m.encode(ids, mask)
    torch.cuda.synchronize()
    assert torch.equal(y, y2)
    # each chunk = its sequences encoded alone (no split applies to either alone)
    assert m._split_point(n1, L) == 0 and m._split_point(B - n1, L) == 0
    assert torch.equal(y[:n1], m.encode(ids[:n1], mask[:n1]))
    assert torch.equal(y[n1:], m.encode(ids[n1:], mask[n1:]))
    m.split_tail = False
    y0 = m.encode(ids, mask)
    err = (y.float() - y0.float()).abs().max().item()
    assert err <= 3e-2 * y0.float().abs().max().item(), err
