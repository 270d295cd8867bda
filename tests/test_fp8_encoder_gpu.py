"""fp8 (e4m3) encoder weights (BASELINE config C5; reference call site: the frozen
BERT of src/contrastor/contrastive_module.py:36-41 -> HF nn.Linear layers).

* irc_quantize_rows_fp8 is bit-exact against oracle.quantize_rows_e4m3 (fp32
  arithmetic, OCP e4m3fn RNE + saturation, itself pinned to torch's cast).
* irc_gemm_fp8 against a torch fp32 reference of the SAME dequantised operands
  (products of e4m3 values are exact in fp32; only the summation order and the
  bf16 output rounding differ).
* MX-fp8 (the encoder's fp8 path since round 3: e4m3 + one E8M0 scale per 32
  values, applied inside v_mfma_scale_f32_16x16x128_f8f6f4): irc_quantize_mx_fp8
  bit-exact against oracle.quantize_mx_e4m3; irc_gemm_mx against the fp64 product
  of the oracle-dequantised operands with block scales spread over 2^-20..2^20
  (a scale applied to the wrong k-block / row / column is off by orders of
  magnitude); the fused producers (LayerNorm, attention, the GEMM's GELU epilogue)
  bit-exact against quantising the bf16 output of their bf16 forms.
* The fp8 BERT-base forward against the reference's fp32 HF output
  (tests/golden/bert_base.npz) by tolerance: the error of e4m3 weights and
  inputs is stated and bounded: on MI355X rms 7.1e-2 on O(1) LayerNorm outputs
  after 12 layers, pooled seq2vec cosine 0.998 (asserted: rms <= 0.1, cosine
  >= 0.995).
"""
import numpy as np
import pytest
import torch

import synth_inputs as SI
from conftest import load_golden
from oracle import irc_oracle as O

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_quantize_rows_bit_exact(gpu, dtype):
    from irc_amd import ops

    g = torch.Generator().manual_seed(3)
    x = (torch.randn(300, 768, generator=g) * torch.logspace(-3, 2, 300)[:, None]).to(dtype)
    x[7] = 0  # zero row -> scale 1
    x[9, 5] = 1e4  # one outlier row
    q, s = ops.quantize_rows_fp8(x.to(gpu))
    rq, rs = O.quantize_rows_e4m3(x.float().numpy())
    np.testing.assert_array_equal(q.cpu().numpy(), rq)
    np.testing.assert_array_equal(s.cpu().numpy(), rs)


@pytest.mark.parametrize("epi", [0, 1, 2, 3])
@pytest.mark.parametrize("M,N,K", [(512, 768, 768), (300, 2304, 768), (1000, 768, 3072)])
def test_gemm_fp8_vs_torch(gpu, epi, M, N, K):
    from irc_amd import ops

    g = torch.Generator().manual_seed(M + N + K + epi)
    a = torch.randn(M, K, generator=g).to(gpu)
    w = (torch.randn(N, K, generator=g) * 0.02).to(gpu)
    bias = (torch.randn(N, generator=g) * 0.1).to(gpu)
    res = torch.randn(M, N, generator=g).bfloat16().to(gpu)
    aq, sa = ops.quantize_rows_fp8(a)
    wq, sw = ops.quantize_rows_fp8(w)
    out = ops.gemm_fp8(aq, sa, wq, sw, bias=bias if epi else None, epilogue=epi,
                       residual=res if epi == 3 else None).float()
    deq = lambda q, s: torch.from_numpy(O.dequantize_e4m3(q.cpu().numpy())).to(gpu) * s[:, None]  # noqa: E731
    ref = deq(aq, sa) @ deq(wq, sw).T
    if epi:
        ref = ref + bias
    if epi == 2:
        ref = torch.nn.functional.gelu(ref)
    if epi == 3:
        ref = ref + res.float()
    err = (out - ref).abs()
    assert bool((err <= 8e-3 * ref.abs() + 2e-3).all()), err.max().item()


def test_bert_base_fp8_weights_vs_reference(gpu):
    from irc_amd.bert import BertConfig, BertModel

    g = load_golden("bert_base.npz")
    m = BertModel(BertConfig(**SI.BERT_BASE))
    sd = {n: torch.from_numpy(SI.bert_param(n, tuple(v.shape)))
          for n, v in m.state_dict().items() if "position_ids" not in n}
    m.load_state_dict(sd, strict=False)
    m = m.to(gpu)
    m.set_weight_format("fp8")
    out = m.encode(torch.from_numpy(g["input_ids"]).to(gpu),
                   torch.from_numpy(g["attention_mask"]).to(gpu)).float().cpu().numpy()
    ref = g["last_hidden_state"]
    err = np.abs(out - ref).max()
    rms = np.sqrt(np.mean((out - ref) ** 2))
    pooled = out.astype(np.float64).mean(axis=1)
    pooled /= np.linalg.norm(pooled, axis=1, keepdims=True)
    cos = (pooled * g["seq2vec"]).sum(axis=1)
    print(f"BERT-base fp8 weights: max abs err {err:.3e}, rms {rms:.3e}, pooled cosine "
          f"{cos.min():.6f}")
    assert np.isfinite(out).all()
    assert rms <= 0.1 and cos.min() >= 0.995


def _mx_matrix(gen, M, K, spread=20):
    """[M, K] fp32 whose 32-value blocks have wildly different magnitudes."""
    x = torch.randn(M, K, generator=gen)
    mag = torch.pow(2.0, torch.randint(-spread, spread + 1, (M, K // 32), generator=gen).float())
    return x * mag.repeat_interleave(32, dim=1)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_quantize_mx_bit_exact(gpu, dtype):
    from irc_amd import ops

    g = torch.Generator().manual_seed(5)
    x = _mx_matrix(g, 300, 768).to(dtype)
    x[7, :32] = 0          # zero block -> scale 2^0
    x[9, 64:96] = 448.0    # exactly at the e4m3 maximum -> scale 2^0
    x[9, 96:128] = 448.25  # just above -> scale 2^1
    mx = ops.quantize_mx(x.to(gpu))
    rc, rs = O.quantize_mx_e4m3(x.float().numpy())
    np.testing.assert_array_equal(mx.codes.cpu().numpy(), rc)
    np.testing.assert_array_equal(mx.scales.cpu().numpy(), rs)


@pytest.mark.parametrize("epi", [0, 1, 2, 3])
@pytest.mark.parametrize("M,N,K", [(300, 384, 512), (1024, 768, 768), (260, 2304, 1024)])
def test_gemm_mx_vs_oracle(gpu, epi, M, N, K):
    from irc_amd import ops

    g = torch.Generator().manual_seed(M + N + K + epi)
    a = _mx_matrix(g, M, K)
    w = _mx_matrix(g, N, K)
    bias = torch.randn(N, generator=g)
    res = torch.randn(M, N, generator=g).bfloat16()
    am, wm = ops.quantize_mx(a.to(gpu)), ops.quantize_mx(w.to(gpu))
    A = O.dequantize_mx_e4m3(am.codes.cpu().numpy(), am.scales.cpu().numpy())
    W = O.dequantize_mx_e4m3(wm.codes.cpu().numpy(), wm.scales.cpu().numpy())
    ref = A @ W.T  # exact products; fp64 sums
    scale = np.abs(A) @ np.abs(W).T  # the fp32-accumulation error scale
    out = ops.gemm_mx(am, wm, bias=bias.to(gpu) if epi else None, epilogue=epi,
                      residual=res.to(gpu) if epi == 3 else None).float().cpu().numpy()
    if epi:
        ref = ref + bias.double().numpy()
        scale = scale + np.abs(bias.double().numpy())
    if epi == 2:
        ref = torch.nn.functional.gelu(torch.from_numpy(ref)).numpy()
    if epi == 3:
        ref = ref + res.double().numpy()
        scale = scale + np.abs(res.double().numpy())
    # bf16 output rounding + fp32 accumulation of terms spanning 2^80 (blocks scaled
    # 2^-20..2^20 on both sides): 1e-4 of the |A||W| scale; a scale applied to the
    # wrong block / row / column is wrong by orders of magnitude
    err = np.abs(out - ref)
    bad = err > 4e-3 * np.abs(ref) + 1e-4 * scale + 1e-30
    worst = (err / (np.abs(ref) + 1e-4 * scale)).max()
    print(f"gemm_mx M={M} N={N} K={K} epi={epi}: worst err / (|ref| + 1e-4 scale) {worst:.3e}")
    assert not bad.any(), worst


@pytest.mark.parametrize("epi", [1, 2])
def test_gemm_mx_output_equals_quantised_bf16(gpu, epi):
    """FFN1's MX epilogue: the e4m3 output + scales equal quantize_mx of the same
    GEMM's bf16 output, bit for bit."""
    from irc_amd import ops

    g = torch.Generator().manual_seed(11 + epi)
    M, N, K = 700, 3072, 768
    am = ops.quantize_mx(torch.randn(M, K, generator=g).to(gpu))
    wm = ops.quantize_mx((torch.randn(N, K, generator=g) * 0.03).to(gpu))
    bias = (torch.randn(N, generator=g) * 0.1).to(gpu)
    y = ops.gemm_mx(am, wm, bias=bias, epilogue=epi)
    ym = ops.gemm_mx(am, wm, bias=bias, epilogue=epi, out_mx=True)
    ref = ops.quantize_mx(y)
    assert torch.equal(ym.codes, ref.codes)
    assert torch.equal(ym.scales, ref.scales)


@pytest.mark.parametrize("H", [768, 1024])
def test_layernorm_mx_equals_quantised_layernorm(gpu, H):
    from irc_amd import ops

    g = torch.Generator().manual_seed(H)
    x = (torch.randn(1000, H, generator=g) * 3).bfloat16().to(gpu)
    gam = (1 + 0.1 * torch.randn(H, generator=g)).to(gpu)
    bet = (0.1 * torch.randn(H, generator=g)).to(gpu)
    y = ops.layernorm(x, gam, bet, 1e-12)
    y2, ym = ops.layernorm_mx(x, gam, bet, 1e-12)
    assert torch.equal(y, y2)
    ref = ops.quantize_mx(y)
    assert torch.equal(ym.codes, ref.codes) and torch.equal(ym.scales, ref.scales)


@pytest.mark.parametrize("L", [64, 72, 17, 129, 200, 512])
def test_attention_mx_equals_quantised_attention(gpu, L):
    from irc_amd import ops

    g = torch.Generator().manual_seed(17 + L)
    B, H, heads = 9, 768, 12
    qkv = torch.randn(B * L, 3 * H, generator=g).bfloat16().to(gpu)
    mask = torch.ones(B, L, dtype=torch.int64)
    mask[3, min(40, L - 1):] = 0
    mask[5, 1:] = 0
    mask = mask.to(gpu)
    ctx = ops.attention(qkv, mask, B, L, H, heads)
    cm = ops.attention_mx(qkv, mask, B, L, H, heads)
    ref = ops.quantize_mx(ctx)
    assert torch.equal(cm.codes, ref.codes) and torch.equal(cm.scales, ref.scales)
