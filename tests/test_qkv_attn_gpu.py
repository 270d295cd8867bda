"""irc_qkv_attention (QKV projection + self-attention in one launch) vs the two-launch
form (irc_gemm EPI_BIAS + irc_attention) and a plain PyTorch fp32 reference.

HF BertSelfAttention as the frozen encoder reaches it (contrastive_module.py:36-41 ->
modeling_bert): softmax(Q K^T / 8 + (1 - mask) * min) V per head, head dim 64, L <= 64
(one 64-row slot per sequence: the joint padding of a batch lands on any L).
Where the unfused QKV GEMM runs on the same big-tile main loop (N = 3H = 2304 at
M = 32768), the fused context must equal the unfused one bit for bit; elsewhere both are
held to the fp32 reference (bf16 operands: the fused error within 1.5x of the unfused
one plus a small floor)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _inputs(gpu, B, L, H, seed, masked=True):
    g = torch.Generator().manual_seed(seed)
    x = (torch.randn(B * L, H, generator=g) * 0.5).bfloat16().to(gpu)
    w = (torch.randn(3 * H, H, generator=g) * 0.05).bfloat16().to(gpu)
    b = (torch.randn(3 * H, generator=g) * 0.1).to(gpu)
    mask = torch.ones(B, L, dtype=torch.int64)
    if masked:
        lens = torch.randint(1, L + 1, (B,), generator=g)
        mask = (torch.arange(L)[None, :] < lens[:, None]).to(torch.int64)
    return x, w, b, mask.to(gpu)


def _ref(x, w, b, mask, B, L, H, heads):
    qkv = x.float() @ w.float().T + b
    q, k, v = (t.view(B, L, heads, 64).transpose(1, 2) for t in qkv.split(H, dim=1))
    bias = (1.0 - mask.float())[:, None, None, :] * torch.finfo(torch.float32).min
    p = torch.softmax(q @ k.transpose(-1, -2) / 8.0 + bias, -1)
    return (p @ v).transpose(1, 2).reshape(B * L, H)


def _fused(x, w, b, mask, B, L, H, heads):
    from irc_amd import ops

    perm = ops.qkv_perm_index(H, x.device)
    return ops.qkv_attention(x, w.index_select(0, perm).contiguous(),
                             b.index_select(0, perm).contiguous(), mask, B, L, H, heads)


def _unfused(x, w, b, mask, B, L, H, heads):
    from irc_amd import ops

    qkv = ops.gemm(x, w, bias=b, epilogue=ops.EPI_BIAS)
    return ops.attention(qkv, mask, B, L, H, heads)


def test_perm_index():
    from irc_amd import ops

    p = ops.qkv_perm_index(768)
    assert sorted(p.tolist()) == list(range(3 * 768))
    # block 1 = Q rows 128..255, K rows 768+128.., V rows 1536+128..
    assert p[384:512].tolist() == list(range(128, 256))
    assert p[512:640].tolist() == list(range(768 + 128, 768 + 256))
    assert p[640:768].tolist() == list(range(1536 + 128, 1536 + 256))


@pytest.mark.parametrize("masked,L", [(True, 64), (False, 64), (True, 63), (True, 57),
                                      (False, 61), (True, 40), (True, 72), (True, 100),
                                      (False, 128), (True, 128), (True, 32), (True, 48),
                                      (False, 51), (True, 65), (True, 80), (False, 85),
                                      (True, 29), (False, 31), (True, 96)])
def test_bit_exact_on_big_tile_shape(gpu, masked, L):
    """B x L ~ 32k rows, where the unfused QKV GEMM runs on the big-tile main loop
    (L <= 64: 64-row slots, four sequences a tile; L in (64, 128]: 128-row slots, two;
    packed tiles of 256 // L sequences, staged a head at a time, where they take fewer
    waves: e.g. L = 40 / 48 / 65 / 72 / 80 / 85 here)."""
    B = {40: 800, 72: 448, 100: 320, 128: 256}.get(L, 512 if 52 <= L <= 64 else 32768 // L)
    H, heads = 768, 12
    x, w, b, mask = _inputs(gpu, B, L, H, 5, masked)
    cf = _fused(x, w, b, mask, B, L, H, heads)
    cu = _unfused(x, w, b, mask, B, L, H, heads)
    assert torch.equal(cf, cu)
    ref = _ref(x, w, b, mask, B, L, H, heads)
    assert (cf.float() - ref).norm() / ref.norm() < 1e-2


@pytest.mark.parametrize("B,H,heads,L", [(37, 768, 12, 64), (4, 768, 12, 64), (64, 1024, 16, 64),
                                         (37, 768, 12, 40), (5, 768, 12, 1), (64, 1024, 16, 50),
                                         (300, 768, 12, 48), (9, 768, 12, 17),
                                         (37, 768, 12, 72), (3, 768, 12, 100),
                                         (33, 1024, 16, 128), (7, 768, 12, 65),
                                         (5, 768, 12, 85), (11, 1024, 16, 33),
                                         (37, 768, 12, 30), (3, 1024, 16, 32)])
def test_against_reference(gpu, B, H, heads, L):
    """Ragged last tile (B = 37: 2368 rows), a single partial tile, BERT-large width;
    L < 64 (slots with repeated last tokens: B = 37 at L = 40 leaves a 1-sequence last
    tile, L = 1 a single key); packed tiles (B = 37 at L = 30: eight sequences a tile, five
    in the last; B = 3 at L = 32: one partial tile)."""
    x, w, b, mask = _inputs(gpu, B, L, H, B + H)
    cf = _fused(x, w, b, mask, B, L, H, heads).float()
    cu = _unfused(x, w, b, mask, B, L, H, heads).float()
    ref = _ref(x, w, b, mask, B, L, H, heads)
    ef = (cf - ref).abs().max().item()
    eu = (cu - ref).abs().max().item()
    assert ef <= 1.5 * eu + 2e-3 * ref.abs().max().item(), (ef, eu)
    assert (cf - ref).norm() / ref.norm() < 1e-2


def test_rejects_unsupported(gpu):
    from irc_amd import ops

    x, w, b, mask = _inputs(gpu, 4, 129, 768, 1)
    with pytest.raises(ValueError):
        _fused(x, w, b, mask, 4, 129, 768, 12)  # L = 129
    x, w, b, mask = _inputs(gpu, 4, 64, 768, 1)
    with pytest.raises(TypeError):
        ops.qkv_attention(x.float(), w, b, mask, 4, 64, 768, 12)


@pytest.mark.parametrize("L", [64, 61, 120, 32, 80])
def test_encoder_fused_matches_unfused(gpu, L):
    """The frozen encoder with the fused launch equals the two-launch encoder bit for bit
    where every unfused QKV GEMM runs on the big-tile main loop: L = 64 and a joint padding
    of 61 (slots), L = 120 at B = 256 (128-row slots), L = 32 and 80 at B = 512 (packed)."""
    import dataclasses

    from irc_amd.bert import BERT_BASE, BertModel

    cfg = dataclasses.replace(BERT_BASE, num_hidden_layers=2)
    m = BertModel(cfg, seed=4).to(gpu)
    g = torch.Generator().manual_seed(2)
    B = {120: 256}.get(L, 512)
    ids = torch.randint(1, cfg.vocab_size, (B, L), generator=g)
    lens = torch.randint(8, L + 1, (B,), generator=g)
    mask = (torch.arange(L)[None, :] < lens[:, None]).to(torch.int64)
    ids[mask == 0] = 0
    ids, mask = ids.to(gpu), mask.to(gpu)
    m.fused_attention = False
    y0 = m.encode(ids, mask)
    m.fused_attention = True
    y1 = m.encode(ids, mask)
    assert torch.equal(y0, y1)


@pytest.mark.parametrize("L", [64, 32, 80, 120])
def test_bit_exact_masks_with_holes(gpu, L):
    """Masks with holes, a lone late key, a lone first key and all-masked rows (the
    epilogue skips key blocks past a sequence's last visible key, as irc_attention
    does): fused equals two-launch bit for bit (slots at 64 / 120, packed at 32 / 80)."""
    B = {64: 512, 120: 256}.get(L, 32768 // L)
    H, heads = 768, 12
    x, w, b, _ = _inputs(gpu, B, L, H, 9, masked=False)
    g = torch.Generator().manual_seed(L)
    kind = torch.randint(0, 5, (B,), generator=g)
    lens = torch.randint(1, L + 1, (B,), generator=g)
    pos = torch.arange(L)[None, :]
    mask = torch.where((kind == 0)[:, None], (pos < lens[:, None]), torch.zeros(1, L, dtype=torch.bool))
    mask |= (kind == 1)[:, None] & ((pos % 7) == (lens[:, None] % 7))   # holes
    mask |= (kind == 2)[:, None] & (pos == L - 1)                         # lone last key
    mask |= (kind == 3)[:, None] & (pos == 0)                             # lone first key
    mask = mask.to(torch.int64).to(gpu)                                    # kind 4: all masked
    cf = _fused(x, w, b, mask, B, L, H, heads)
    cu = _unfused(x, w, b, mask, B, L, H, heads)
    assert torch.equal(cf, cu)
