"""Whole-wave splits.  The frozen encoder's split form (irc_amd.bert.BertModel._encode_split): a batch whose
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


def test_head_input_projection_split(gpu):
    """The LSTM head's input projection at B L = 256 x 65 rows (irc_amd.lstm_head.
    _gemm_rows_split): the whole-wave rows on the calling stream equal the one-launch
    GEMM bit for bit (same 256 x 256 tiles), the 256 tail rows on the side stream agree
    within fp32 reassociation (a smaller launch takes another kernel)."""
    from irc_amd import lstm_head, ops

    g = torch.Generator().manual_seed(3)
    M, K, N = 256 * 65, 768, 2048
    x = (torch.randn(M, K, generator=g) * 0.5).bfloat16().to(gpu)
    w = (torch.randn(N, K, generator=g) / K ** 0.5).bfloat16().to(gpu)
    b = torch.randn(N, generator=g).to(gpu)
    ref = ops.gemm(x, w, bias=b, epilogue=ops.EPI_BIAS, out_dtype=torch.float32)
    got = lstm_head._gemm_rows_split(x, w, b)
    torch.cuda.synchronize()
    full = M // 8192 * 8192
    assert full == 16384
    assert torch.equal(got[:full], ref[:full])
    assert torch.allclose(got[full:], ref[full:], rtol=1e-5, atol=1e-5)
