"""irc_attention vs a plain PyTorch fp32 reference of the same op: HF BertSelfAttention
in eval mode (modeling_bert, reached from contrastive_module.py:39):
softmax(Q K^T / sqrt(dh) + (1 - mask) * finfo.min) V over the fused [B*L, 3H] QKV rows.

bf16 with head dim 64 runs an MFMA kernel at every L the reference's tokenizer can
produce (joint padding up to 512, contrastive_module.py:38): whole score rows in
registers for L <= 128 (L not a multiple of 32, e.g. a joint-padded batch's L = 72:
clamped key rows with a pad bias, zero V rows, query rows past L never stored), keys
streamed with an online softmax above; other shapes / fp32 run the key-tiled VALU
kernel, also at any L.  Tolerance: bf16 -> ATT_ULPS bf16 ulps of the reference value,
the ulp taken at max(|ref|, ATT_FLOOR) (conftest.bf16_ulps: the bf16 inputs, the
bf16-rounded probabilities and the bf16 output); fp32 -> 1e-5 absolute.
"""
import pytest
import torch

from conftest import bf16_ulps

pytestmark = pytest.mark.gpu

ATT_FLOOR = 0.5  # the context's scale: averages of V rows ~ N(0, 1)
ATT_ULPS = 3.0  # measured on MI355X: at most 1.52 over L in [1, 512] (r6_b)


def _ref(qkv, mask, B, L, H, heads):
    dh = H // heads
    x = qkv.float().cpu().view(B, L, 3, heads, dh)
    q, k, v = (x[:, :, i].permute(0, 2, 1, 3) for i in range(3))  # [B, heads, L, dh]
    s = q @ k.transpose(-1, -2) / dh ** 0.5
    bias = (1.0 - mask.cpu().float())[:, None, None, :] * torch.finfo(torch.float32).min
    p = torch.softmax(s + bias, dim=-1)
    return (p @ v).permute(0, 2, 1, 3).reshape(B * L, H)


def _case(B, L, H, heads, dtype, seed, all_masked_row=False):
    g = torch.Generator().manual_seed(seed)
    qkv = torch.randn((B * L, 3 * H), generator=g).to(dtype)
    lens = torch.randint(1, L + 1, (B,), generator=g)
    lens[0] = L
    mask = (torch.arange(L)[None, :] < lens[:, None]).long()
    if all_masked_row:
        mask[-1] = 0
    return qkv, mask


@pytest.mark.parametrize("L", [1, 17, 32, 40, 64, 72, 93, 96, 100, 128,
                               129, 160, 200, 317, 318, 400, 512])
def test_attention_mfma_bf16(gpu, L):
    from irc_amd import ops

    B, H, heads = 5, 768, 12
    qkv, mask = _case(B, L, H, heads, torch.bfloat16, L, all_masked_row=True)
    out = ops.attention(qkv.to(gpu), mask.to(gpu), B, L, H, heads)
    ref = _ref(qkv, mask, B, L, H, heads)
    assert torch.isfinite(out.float()).all()
    # bf16 context (|ref| <~ 3, V ~ N(0, 1)): P and the output rounded to bf16
    e = bf16_ulps(out.float().cpu().numpy(), ref.numpy(), ATT_FLOOR)
    print(f"L={L}: {e:.2f} bf16 ulps")
    assert e <= ATT_ULPS, f"{e:.2f} bf16 ulps"


@pytest.mark.parametrize("dtype,L,H,heads", [(torch.float32, 64, 768, 12),
                                             (torch.bfloat16, 40, 768, 12),
                                             (torch.bfloat16, 64, 256, 8),
                                             (torch.float32, 17, 128, 2),
                                             (torch.float32, 300, 768, 12),
                                             (torch.float32, 512, 32, 2),
                                             (torch.bfloat16, 257, 256, 8)])
def test_attention_valu_shapes(gpu, dtype, L, H, heads):
    from irc_amd import ops

    B = 3
    qkv, mask = _case(B, L, H, heads, dtype, 11 * L + H, all_masked_row=True)
    out = ops.attention(qkv.to(gpu), mask.to(gpu), B, L, H, heads)
    ref = _ref(qkv, mask, B, L, H, heads)
    if dtype == torch.float32:
        assert (out.float().cpu() - ref).abs().max().item() <= 1e-5
    else:
        e = bf16_ulps(out.float().cpu().numpy(), ref.numpy(), ATT_FLOOR)
        assert e <= ATT_ULPS, f"{e:.2f} bf16 ulps"


def test_attention_long_rows_all_masked_and_single_key(gpu):
    """L = 512 with an all-masked row (uniform average over all 512 keys, HF's finfo.min
    bias) and a row whose only unmasked key is the last one (online-softmax rescale
    across 16 key tiles)."""
    from irc_amd import ops

    B, L, H, heads = 3, 512, 768, 12
    g = torch.Generator().manual_seed(512)
    qkv = torch.randn((B * L, 3 * H), generator=g)
    qkv[:, :2 * H] *= 3  # peaked softmax rows: the running max moves between key tiles
    qkv = qkv.bfloat16()
    mask = torch.ones(B, L, dtype=torch.int64)
    mask[1] = 0
    mask[2, :-1] = 0
    out = ops.attention(qkv.to(gpu), mask.to(gpu), B, L, H, heads)
    ref = _ref(qkv, mask, B, L, H, heads)
    e = bf16_ulps(out.float().cpu().numpy(), ref.numpy(), ATT_FLOOR)
    print(f"long rows: {e:.2f} bf16 ulps")
    assert e <= ATT_ULPS, f"{e:.2f} bf16 ulps"


@pytest.mark.parametrize("L", [64, 72, 96, 128])
def test_attention_masks_with_holes(gpu, L):
    """Key blocks past a sequence's last visible key are skipped (encoder.hip
    visible_key_blocks): rows whose only visible keys sit late after masked ones, a
    visible key alone in the last block, one alone at position 0, an all-masked row
    (every block kept: the uniform average) -- all against the fp32 reference."""
    from irc_amd import ops

    B, H, heads = 6, 768, 12
    g = torch.Generator().manual_seed(100 + L)
    qkv = torch.randn((B * L, 3 * H), generator=g).bfloat16()
    mask = torch.zeros(B, L, dtype=torch.int64)
    mask[0] = 1                      # all visible
    mask[1, 0] = 1                   # only the first key
    mask[2, L - 1] = 1               # only the last key (last block)
    mask[3, ::5] = 1                 # holes in every block
    mask[4, 3:40] = 1                # a window straddling blocks 0 and 1
    # row 5 all masked
    out = ops.attention(qkv.to(gpu), mask.to(gpu), B, L, H, heads)
    ref = _ref(qkv, mask, B, L, H, heads)
    e = bf16_ulps(out.float().cpu().numpy(), ref.numpy(), ATT_FLOOR)
    print(f"L={L} holes: {e:.2f} bf16 ulps")
    assert e <= ATT_ULPS, f"{e:.2f} bf16 ulps"


def test_attention_skipped_blocks_bit_identical(gpu):
    """Sequences whose visible keys all lie in the first 32: their first 32 context rows
    at L = 64 (the second key block skipped) equal those at L = 32 bit for bit -- the
    skipped block would have added exact zeros -- as they do at L = 96 and 128."""
    from irc_amd import ops

    B, H, heads = 9, 768, 12
    g = torch.Generator().manual_seed(7)
    qkv = torch.randn((B, 128, 3 * H), generator=g).bfloat16()
    lens = torch.randint(1, 33, (B,), generator=g)
    mask = (torch.arange(128)[None, :] < lens[:, None]).long()
    outs = {}
    for L in (32, 64, 96, 128):
        q = qkv[:, :L].reshape(B * L, 3 * H).contiguous().to(gpu)
        m = mask[:, :L].contiguous().to(gpu)
        outs[L] = ops.attention(q, m, B, L, H, heads).view(B, L, H)[:, :32].cpu()
    for L in (64, 96, 128):
        assert torch.equal(outs[L], outs[32]), L
