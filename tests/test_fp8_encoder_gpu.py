"""fp8 (e4m3) encoder weights (BASELINE config C5; reference call site: the frozen
BERT of src/contrastor/contrastive_module.py:36-41 -> HF nn.Linear layers).

* irc_quantize_rows_fp8 is bit-exact against oracle.quantize_rows_e4m3 (fp32
  arithmetic, OCP e4m3fn RNE + saturation, itself pinned to torch's cast).
* irc_gemm_fp8 against a torch fp32 reference of the SAME dequantised operands
  (products of e4m3 values are exact in fp32; only the summation order and the
  bf16 output rounding differ).
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
