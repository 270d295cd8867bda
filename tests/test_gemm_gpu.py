"""irc_gemm (bf16 and exact-fp32 MFMA) vs a plain PyTorch fp32 reference of the same op."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _ref(a, b, trans_a, b_is_nk, bias, epi, res, alpha):
    A = a.float().cpu()
    B = b.float().cpu()
    A = A.t() if trans_a else A
    B = B.t() if b_is_nk else B
    y = alpha * (A @ B)
    if bias is not None:
        y = y + bias.cpu()
    if epi == 2:
        y = torch.nn.functional.gelu(y)
    if res is not None:
        y = y + res.float().cpu()
    return y


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("trans_a,b_is_nk", [(False, True), (False, False), (True, True),
                                             (True, False)])
@pytest.mark.parametrize("M,N,K", [(1, 1, 8), (37, 70, 24), (200, 300, 136), (256, 128, 768)])
def test_layouts(gpu, dtype, trans_a, b_is_nk, M, N, K):
    from irc_amd import ops

    g = torch.Generator().manual_seed(M * 1000 + N + K)
    a = torch.randn((K, M) if trans_a else (M, K), generator=g).to(dtype)
    b = torch.randn((N, K) if b_is_nk else (K, N), generator=g).to(dtype)
    out = ops.gemm(a.to(gpu), b.to(gpu), trans_a=trans_a, b_is_nk=b_is_nk,
                   out_dtype=torch.float32)
    ref = _ref(a, b, trans_a, b_is_nk, None, 0, None, 1.0)
    tol = 1e-4 * K if dtype == torch.float32 else 2e-2 * K ** 0.5
    assert (out.cpu() - ref).abs().max().item() <= tol


@pytest.mark.parametrize("epi", [1, 2, 3, 4])
@pytest.mark.parametrize("odt", [torch.bfloat16, torch.float32])
def test_epilogues(gpu, epi, odt):
    from irc_amd import ops

    g = torch.Generator().manual_seed(epi)
    M, N, K = 300, 260, 192
    a = torch.randn(M, K, generator=g).bfloat16()
    b = torch.randn(N, K, generator=g).bfloat16()
    bias = torch.randn(N, generator=g) if epi in (1, 2, 3) else None
    res = torch.randn(M, N, generator=g).to(odt) if epi in (3, 4) else None
    out = ops.gemm(a.to(gpu), b.to(gpu), bias=None if bias is None else bias.to(gpu),
                   epilogue=epi, residual=None if res is None else res.to(gpu), out_dtype=odt,
                   alpha=0.5)
    ref = _ref(a, b, False, True, bias, epi, res, 0.5)
    rel = (out.float().cpu() - ref).abs().max().item() / ref.abs().max().item()
    assert rel < (1e-2 if odt == torch.bfloat16 else 2e-3)


def test_fp32_accumulate(gpu):
    from irc_amd import ops

    g = torch.Generator().manual_seed(9)
    a = torch.randn(64, 96, generator=g)
    b = torch.randn(80, 96, generator=g)
    c0 = torch.randn(64, 80, generator=g)
    c = c0.clone().to(gpu)
    ops.gemm(a.to(gpu), b.to(gpu), out=c, accumulate=True)
    torch.testing.assert_close(c.cpu(), c0 + a @ b.t(), rtol=1e-5, atol=1e-4)


def test_fp32_mfma_is_exact_on_integers(gpu):
    """exact fp32 products: integer operands give the exact integer result."""
    from irc_amd import ops

    g = torch.Generator().manual_seed(3)
    a = torch.randint(-50, 50, (129, 64), generator=g).float()
    b = torch.randint(-50, 50, (33, 64), generator=g).float()
    out = ops.gemm(a.to(gpu), b.to(gpu)).cpu()
    assert torch.equal(out, a @ b.t())


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("M,N,K", [(1024, 256, 16384), (200, 72, 5000), (64, 64, 1030)])
def test_splitk_batched_accumulate(gpu, dtype, M, N, K):
    """Weight-gradient shape (K = B*L >> M, N): the deterministic split-K path,
    batched over two directions with an interleaved A ([K][2M], lda = 2M) and a
    shared B, accumulating into fp32 C.  Bitwise reproducible run to run."""
    from irc_amd import _lib, ops

    code = 0 if dtype == torch.bfloat16 else 1
    assert _lib.load().irc_gemm_workspace(code, 1, 0, M, N, K, 2) > 0 or K < 1024
    g = torch.Generator().manual_seed(K)
    a = torch.randn((K, 2 * M), generator=g).to(dtype)
    b = torch.randn((K, N), generator=g).to(dtype)
    c0 = torch.randn((2, M, N), generator=g)
    out = c0.clone().to(gpu)
    ad, bd = a.to(gpu), b.to(gpu)
    ops.gemm_strided(ad, bd, out, M=M, N=N, K=K, batch=2, lda=2 * M, sA=M, ldb=N, sB=0, ldc=N,
                     sC=M * N, trans_a=True, b_is_nk=False, accumulate=True)
    af, bf = a.float(), b.float()
    for d in range(2):
        ref = c0[d] + af[:, d * M:(d + 1) * M].t().double().matmul(bf.double()).float()
        tol = 1e-5 * K if dtype == torch.float32 else 1e-4 * K
        assert (out[d].cpu() - ref).abs().max().item() <= tol, d
    out2 = c0.clone().to(gpu)
    ops.gemm_strided(ad, bd, out2, M=M, N=N, K=K, batch=2, lda=2 * M, sA=M, ldb=N, sB=0, ldc=N,
                     sC=M * N, trans_a=True, b_is_nk=False, accumulate=True)
    assert torch.equal(out, out2)


@pytest.mark.parametrize("max_blocks", [0, 32, 128, 1])
def test_splitk_block_cap(gpu, max_blocks):
    """irc_gemm_ex with a split-K cap (the LSTM head's side-stream dW GEMMs: dgates^T . x,
    K = B*L): within fp32 reassociation of the uncapped GEMM, bitwise reproducible, and
    a smaller cap never needs more workspace."""
    from irc_amd import _lib, ops

    M, N, K = 1024, 768, 16640
    lib = _lib.load()
    full = lib.irc_gemm_workspace_ex(0, 1, 0, M, N, K, 2, 0)
    assert full == lib.irc_gemm_workspace(0, 1, 0, M, N, K, 2) > 0
    assert lib.irc_gemm_workspace_ex(0, 1, 0, M, N, K, 2, max_blocks) <= full
    g = torch.Generator().manual_seed(11)
    a = torch.randn((K, 2 * M), generator=g).to(torch.bfloat16).to(gpu)
    b = torch.randn((K, N), generator=g).to(torch.bfloat16).to(gpu)
    outs = []
    for mb in (0, max_blocks, max_blocks):
        c = torch.zeros((2, M, N), device=gpu)
        ops.gemm_strided(a, b, c, M=M, N=N, K=K, batch=2, lda=2 * M, sA=M, ldb=N, sB=0, ldc=N,
                         sC=M * N, trans_a=True, b_is_nk=False, accumulate=True, max_blocks=mb)
        outs.append(c)
    assert torch.equal(outs[1], outs[2])
    torch.testing.assert_close(outs[1], outs[0], rtol=1e-5, atol=2e-3)


@pytest.mark.parametrize("max_blocks", [128, 100, 7])
@pytest.mark.parametrize("M,N,K,epi,od", [(16640, 2048, 768, 1, torch.float32),
                                          (4000, 1536, 512, 2, torch.bfloat16),
                                          (3000, 1000, 256, 0, torch.float32)])
def test_grid_cap_bit_identical(gpu, max_blocks, M, N, K, epi, od):
    """irc_gemm_ex with a negative max_blocks (a grid cap) on a launch of more 256 x 256
    tiles than the cap: a static persistent tile loop over -max_blocks workgroups,
    bit-identical to one workgroup per tile."""
    from irc_amd import ops

    g = torch.Generator().manual_seed(M + N)
    a = torch.randn((M, K), generator=g).to(torch.bfloat16).to(gpu)
    w = torch.randn((N, K), generator=g).to(torch.bfloat16).to(gpu)
    bias = torch.randn(N, generator=g).to(gpu)
    kw = dict(bias=bias if epi else None, epilogue=epi, out_dtype=od)
    ref = ops.gemm(a, w, **kw)
    capped = ops.gemm(a, w, max_blocks=-max_blocks, **kw)
    assert torch.equal(ref, capped)


def test_splitk_matches_unsplit(gpu):
    """Same GEMM with and without the workspace: equal within fp32 reassociation."""
    from irc_amd import _lib, ops
    from irc_amd._torch import ptr, stream_ptr

    M, N, K = 256, 128, 8192
    g = torch.Generator().manual_seed(7)
    a = torch.randn((K, M), generator=g).to(torch.bfloat16).to(gpu)
    b = torch.randn((K, N), generator=g).to(torch.bfloat16).to(gpu)
    split = ops.gemm(a, b, trans_a=True, b_is_nk=False, out_dtype=torch.float32)
    plain = torch.empty((M, N), device=gpu)
    _lib.call("irc_gemm", 0, 1, 1, 1, 0, M, N, K, 1.0, ptr(a), M, 0, ptr(b), N, 0, None, 0, None,
              0, 0, ptr(plain), N, 0, 0, 1, None, 0, stream_ptr(a.device))
    assert _lib.load().irc_gemm_workspace(0, 1, 0, M, N, K, 1) > 0
    torch.testing.assert_close(split, plain, rtol=1e-5, atol=1e-3)


@pytest.mark.parametrize("epi", [0, 1, 2, 3, 4])
@pytest.mark.parametrize("out_dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("M,N,K", [(4000, 2100, 640), (4096, 2048, 768), (8000, 1536, 384)])
def test_big_tile_path(gpu, epi, out_dtype, M, N, K):
    """Large-tile global_load_lds path (bf16, A [M][K], B [N][K], K % 64 == 0, >= 128
    tiles; 256x384 when N % 384 == 0 else 256x256), ragged M / N, every fused
    epilogue, vs a torch fp32 reference."""
    from irc_amd import ops

    g = torch.Generator().manual_seed(M + N + K + epi)
    a = (torch.randn((M, K), generator=g) * 0.5).to(torch.bfloat16)
    b = (torch.randn((N, K), generator=g) * 0.5).to(torch.bfloat16)
    bias = torch.randn((N,), generator=g) if epi in (1, 2, 3) else None
    res = torch.randn((M, N), generator=g).to(out_dtype) if epi in (3, 4) else None
    out = ops.gemm(a.to(gpu), b.to(gpu), bias=None if bias is None else bias.to(gpu), epilogue=epi,
                   residual=None if res is None else res.to(gpu), alpha=0.75,
                   out_dtype=out_dtype)
    ref = _ref(a, b, False, True, bias, epi, res, 0.75)
    err = (out.float().cpu() - ref).abs()
    tol = 2e-3 * K ** 0.5 + (2e-2 * ref.abs() if out_dtype == torch.bfloat16 else 0)
    assert (err <= tol).all(), err.max().item()


def test_big_tile_accumulate_fp32(gpu):
    from irc_amd import ops

    M, N, K = 2048, 4096, 1024
    g = torch.Generator().manual_seed(5)
    a = torch.randn((M, K), generator=g).to(torch.bfloat16)
    b = torch.randn((N, K), generator=g).to(torch.bfloat16)
    c0 = torch.randn((M, N), generator=g)
    out = c0.to(gpu)
    ops.gemm(a.to(gpu), b.to(gpu), out=out, accumulate=True)
    ref = c0 + a.float() @ b.float().t()
    assert (out.cpu() - ref).abs().max().item() <= 2e-3 * K ** 0.5


@pytest.mark.parametrize("epi", [0, 1, 2, 3])
@pytest.mark.parametrize("M,N,K", [(32768, 2304, 768), (32768, 768, 3072), (32668, 768, 192),
                                   (32700, 2304, 64)])
def test_big_tile_ring_bitwise(gpu, epi, M, N, K):
    """The big-tile kernel's 4-slot ring of 32-deep K-tiles (three in flight) against
    its 2-slot 64-deep loop: the same MFMAs in the same k order, so the outputs are
    equal bit for bit -- on the BERT-base QKV / FFN2 shapes (the shapes irc_gemm
    sends to the 256 x 384 kernel: whole waves of its tiles), with ragged M, K = 192
    (six ring K-tiles) and K = 64 (two: fewer than the ring's prefetch depth)."""
    from irc_amd import ops

    g = torch.Generator().manual_seed(M + N + K + epi)
    a = torch.randn((M, K), generator=g).to(torch.bfloat16).to(gpu)
    b = torch.randn((N, K), generator=g).to(torch.bfloat16).to(gpu)
    bias = torch.randn((N,), generator=g).to(gpu) if epi in (1, 2, 3) else None
    res = torch.randn((M, N), generator=g).to(torch.bfloat16).to(gpu) if epi == 3 else None
    outs = []
    prev = ops.gemm_set_big_ring(True)
    try:
        for ring in (True, False):
            ops.gemm_set_big_ring(ring)
            outs.append(ops.gemm(a, b, bias=bias, epilogue=epi, residual=res))
        torch.cuda.synchronize()
    finally:
        ops.gemm_set_big_ring(prev)
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("ring", [False, True])
@pytest.mark.parametrize("M,N,K", [(32768, 2304, 768), (32768, 768, 3072), (4000, 2100, 640)])
def test_big_tile_chunk_key_exact(gpu, ring, M, N, K):
    """The big-tile kernel's LDS chunk key ((r >> 1) & 7 since round 4): small-integer
    operands make every product and partial sum exact in fp32, so the output must equal
    the torch product bit for bit -- a chunk stored under one key and read under another
    (a wrong row, k-chunk or slot) changes the result.  Both the 2-slot and the ring
    form, on the BERT QKV / FFN2 shapes (256 x 384 tiles) and a ragged 256 x 256 case."""
    from irc_amd import ops

    g = torch.Generator().manual_seed(M + N + K)
    a = torch.randint(-8, 9, (M, K), generator=g).to(torch.bfloat16)
    b = torch.randint(-8, 9, (N, K), generator=g).to(torch.bfloat16)
    prev = ops.gemm_set_big_ring(ring)
    try:
        out = ops.gemm(a.to(gpu), b.to(gpu), out_dtype=torch.float32)
        torch.cuda.synchronize()
    finally:
        ops.gemm_set_big_ring(prev)
    ref = (a.to(gpu).float() @ b.to(gpu).float().t())  # |sum| <= 64 * K < 2^24: exact
    assert torch.equal(out, ref)


@pytest.mark.parametrize("epi", [0, 1, 2, 3, 4])
@pytest.mark.parametrize("M,N,K", [(32768, 2304, 768), (32768, 768, 3072), (32700, 2304, 192),
                                   (4000, 2100, 640)])
def test_big_tile_mf16_exact(gpu, epi, M, N, K):
    """The big-tile kernel's 16x16x32 form (irc_gemm_set_big_mf16) on the BERT QKV /
    FFN2 shapes, a ragged M and a 256 x 256 case (N % 384 != 0): small-integer
    operands, bias and residual make every sum exact in fp32, so the output equals the
    32x32x16 form's bit for bit (GELU: the same function of the same exact input)."""
    from irc_amd import ops

    g = torch.Generator().manual_seed(M + N + K + epi)
    a = torch.randint(-4, 5, (M, K), generator=g).to(torch.bfloat16).to(gpu)
    b = torch.randint(-4, 5, (N, K), generator=g).to(torch.bfloat16).to(gpu)
    bias = (torch.randint(-8, 9, (N,), generator=g).float() / 4).to(gpu) if epi in (1, 2, 3) else None
    res = torch.randint(-8, 9, (M, N), generator=g).to(torch.bfloat16).to(gpu) if epi in (3, 4) else None
    outs = []
    prev = ops.gemm_set_big_mf16(False)
    try:
        for mf in (False, True):
            ops.gemm_set_big_mf16(mf)
            outs.append(ops.gemm(a, b, bias=bias, epilogue=epi, residual=res,
                                 out_dtype=torch.bfloat16))
            if epi == 0:  # fp32 output too (the LSTM input projection's form)
                outs.append(ops.gemm(a, b, out_dtype=torch.float32))
        torch.cuda.synchronize()
    finally:
        ops.gemm_set_big_mf16(prev)
    half = len(outs) // 2
    for x, y in zip(outs[:half], outs[half:]):
        assert torch.equal(x, y)
    if epi == 0:
        ref = a.float() @ b.float().t()
        assert torch.equal(outs[1], ref)


def test_big_tile_mf16_random_close(gpu):
    """Random bf16 operands: the 16x16x32 and 32x32x16 forms agree within fp32
    reassociation (FFN2 shape, K = 3072, bias + residual)."""
    from irc_amd import ops

    M, N, K = 32768, 768, 3072
    g = torch.Generator().manual_seed(5)
    a = torch.randn((M, K), generator=g).to(torch.bfloat16).to(gpu)
    b = (torch.randn((N, K), generator=g) * 0.03).to(torch.bfloat16).to(gpu)
    bias = torch.randn((N,), generator=g).to(gpu)
    res = torch.randn((M, N), generator=g).to(gpu)
    outs = []
    prev = ops.gemm_set_big_mf16(False)
    try:
        for mf in (False, True):
            ops.gemm_set_big_mf16(mf)
            outs.append(ops.gemm(a, b, bias=bias, epilogue=3, residual=res,
                                 out_dtype=torch.float32))
        torch.cuda.synchronize()
    finally:
        ops.gemm_set_big_mf16(prev)
    assert (outs[0] - outs[1]).abs().max().item() <= 1e-4 * K ** 0.5


@pytest.mark.parametrize("M,N", [(4096, 3072), (32768, 768), (300, 260)])
def test_gelu_bf16_epilogue_matches_exact_erf_gelu(gpu, M, N):
    """The bf16-output GELU epilogue (gelu_lite2, irc_common.h) against torch's exact erf
    GELU of HF BertIntermediate.  A = stacked identities makes the GEMM exact (one
    product per output), so C = GELU(B^T) rounded to bf16: at most 1 bf16 ulp from
    bf16(exact GELU) anywhere, and equal for >= 99% of the elements (the fit's error is
    <= 0.15 ulp wherever |GELU| >= 1e-2)."""
    from irc_amd import ops

    K = 256
    g = torch.Generator().manual_seed(M + N)
    a = torch.eye(K).repeat((M + K - 1) // K, 1)[:M].to(torch.bfloat16)
    b = (torch.randn((N, K), generator=g) * 3).to(torch.bfloat16)
    out = ops.gemm(a.to(gpu), b.to(gpu), bias=torch.zeros(N, device=gpu), epilogue=2,
                   out_dtype=torch.bfloat16).cpu()
    x = b.float().t().repeat((M + K - 1) // K, 1)[:M]
    ref = torch.nn.functional.gelu(x.double()).to(torch.bfloat16)
    oi, ri = out.view(torch.int16).int(), ref.view(torch.int16).int()
    same_sign = (out.float() * ref.float() >= 0)
    ulps = torch.where(same_sign, (oi - ri).abs(), torch.full_like(oi, 1 << 20))
    small = ref.float().abs() < 1e-4  # |GELU| < 1e-4: absolute error bound instead
    assert ((out.float() - ref.float()).abs()[small] <= 1e-5).all()
    assert (ulps[~small] <= 1).all(), ulps[~small].max().item()
    # measured on MI355X: 95.7% exact over |GELU| >= 1e-4; the 1-ulp flips sit mostly
    # where |GELU| < 1e-2 (absolute error < 6e-5 there)
    big = ref.float().abs() >= 1e-2
    assert (ulps[big] == 0).float().mean().item() >= 0.95


# ---- the 256x256 ping-pong path (gemm_pp.hip): shapes with >= 32 output tiles
@pytest.mark.parametrize("trans_a,b_is_nk", [(False, True), (False, False), (True, True),
                                             (True, False)])
@pytest.mark.parametrize("M,N,K", [(2048, 1024, 256), (1800, 1208, 320)])
def test_pp_layouts(gpu, trans_a, b_is_nk, M, N, K):
    """All four operand layouts, ragged M/N (not multiples of 256), bf16 in, fp32 out.
    Tolerance: bf16 operands, fp32 accumulation -> 1e-3 relative to max |ref|."""
    from irc_amd import ops

    g = torch.Generator().manual_seed(M + N + K + 7 * trans_a + 3 * b_is_nk)
    a = torch.randn((K, M) if trans_a else (M, K), generator=g).bfloat16()
    b = torch.randn((N, K) if b_is_nk else (K, N), generator=g).bfloat16()
    out = ops.gemm(a.to(gpu), b.to(gpu), trans_a=trans_a, b_is_nk=b_is_nk,
                   out_dtype=torch.float32)
    ref = _ref(a, b, trans_a, b_is_nk, None, 0, None, 1.0)
    assert (out.cpu() - ref).abs().max().item() <= 1e-3 * ref.abs().max().item()


@pytest.mark.parametrize("epi", [0, 1, 2, 3, 4, 5, 6])
@pytest.mark.parametrize("odt", [torch.bfloat16, torch.float32])
def test_pp_epilogues(gpu, epi, odt):
    from irc_amd import ops

    M, N, K = 2304, 1040, 192
    g = torch.Generator().manual_seed(100 + epi)
    a = torch.randn(M, K, generator=g).bfloat16()
    b = torch.randn(N, K, generator=g).bfloat16()
    bias = torch.randn(N, generator=g) if epi in (1, 2, 3, 6) else None
    res = torch.randn(M, N, generator=g).to(odt) if epi in (3, 4, 5, 6) else None
    out = ops.gemm(a.to(gpu), b.to(gpu), bias=None if bias is None else bias.to(gpu),
                   epilogue=epi, residual=None if res is None else res.to(gpu), out_dtype=odt,
                   alpha=0.5)
    y = 0.5 * (a.float() @ b.float().T)
    if bias is not None:
        y = y + bias
    if epi == 2:
        ref = torch.nn.functional.gelu(y)
    elif epi in (3, 4):
        ref = y + res.float()
    elif epi == 5:
        ur = res.float().requires_grad_(True)
        torch.nn.functional.gelu(ur).backward(y)
        ref = ur.grad
    elif epi == 6:
        ref = torch.nn.functional.gelu(y)
    else:
        ref = y
    tol = 1e-2 if odt == torch.bfloat16 else 1e-3
    assert (out.float().cpu() - ref).abs().max().item() <= tol * ref.abs().max().item()


def test_pp_gelu_save_writes_preactivation(gpu):
    from irc_amd import ops

    M, N, K = 2048, 1024, 128
    g = torch.Generator().manual_seed(5)
    a = torch.randn(M, K, generator=g).bfloat16().to(gpu)
    b = torch.randn(N, K, generator=g).bfloat16().to(gpu)
    bias = torch.randn(N, generator=g).to(gpu)
    out, pre = ops.gemm_gelu_save(a, b, bias)
    y = a.float().cpu() @ b.float().cpu().T + bias.cpu()
    assert (pre.float().cpu() - y).abs().max().item() <= 1e-2 * y.abs().max().item()
    assert (out.float().cpu() - torch.nn.functional.gelu(y)).abs().max().item() <= \
        1e-2 * y.abs().max().item()


@pytest.mark.parametrize("M,N,K,batch", [(768, 768, 16384, 1), (1024, 256, 8192, 2),
                                         (3072, 768, 4096, 1)])
def test_pp_splitk_accumulate(gpu, M, N, K, batch):
    """Weight-gradient shapes: both operands K-outer, few output tiles -> deterministic
    split-K slabs, fp32 accumulate into an existing gradient.  Bitwise repeatable."""
    from irc_amd import ops

    g = torch.Generator().manual_seed(M + K)
    a = torch.randn((batch, K, M), generator=g).bfloat16().to(gpu)
    b = torch.randn((batch, K, N), generator=g).bfloat16().to(gpu)
    base = torch.randn((batch, M, N), generator=g).to(gpu)
    outs = []
    for _ in range(2):
        out = base.clone()
        ops.gemm_strided(a, b, out, M=M, N=N, K=K, batch=batch, lda=M, sA=K * M, ldb=N, sB=K * N,
                         ldc=N, sC=M * N, trans_a=True, b_is_nk=False, accumulate=True)
        outs.append(out)
    assert torch.equal(outs[0], outs[1])
    ref = base.cpu() + torch.einsum("bkm,bkn->bmn", a.float().cpu(), b.float().cpu())
    err = (outs[0].cpu() - ref).abs().max().item()
    assert err <= 1e-3 * ref.abs().max().item()


# ---- persistent form of the 256x256 path: launches of more tiles than CUs
@pytest.mark.parametrize("epi", [0, 1, 2, 3, 4, 5, 6])
@pytest.mark.parametrize("odt", [torch.bfloat16, torch.float32])
def test_pp_persistent_bitwise(gpu, epi, odt):
    """17 x 17 = 289 ragged output tiles (> 256 CUs): the persistent tile loop
    (dynamic tile counter, next tile's first K-tile DMA'd during the epilogue) gives
    the same bits as one workgroup per tile, for every epilogue, and matches the
    fp32 reference within the bf16 tolerance of test_pp_epilogues."""
    from irc_amd import ops

    M, N, K = 4100, 4200, 192
    g = torch.Generator().manual_seed(300 + epi)
    a = torch.randn(M, K, generator=g).bfloat16()
    b = torch.randn(N, K, generator=g).bfloat16()
    bias = torch.randn(N, generator=g) if epi in (1, 2, 3, 6) else None
    res = torch.randn(M, N, generator=g).to(odt) if epi in (3, 4, 5, 6) else None
    outs = []
    prev = ops.gemm_set_persistent(True)
    try:
        # modes: 1 dynamic tiles (twice: the tile counter resets), 0 one workgroup per
        # tile, 2 static waves + prestage, 3 static without prestage
        for pers in (1, 0, 1, 2, 3):
            ops.gemm_set_persistent(pers)
            r = None if res is None else res.to(gpu)
            out = ops.gemm(a.to(gpu), b.to(gpu), bias=None if bias is None else bias.to(gpu),
                           epilogue=epi, residual=r, out_dtype=odt, alpha=0.5)
            torch.cuda.synchronize()
            outs.append((out.cpu(), None if r is None else r.cpu()))
    finally:
        ops.gemm_set_persistent(prev)
    for o, r in outs[1:]:
        assert torch.equal(o, outs[0][0])
        if epi == 6:  # pre-activation written to R
            assert torch.equal(r, outs[0][1])
    y = 0.5 * (a.float() @ b.float().T)
    if bias is not None:
        y = y + bias
    if epi in (2, 6):
        ref = torch.nn.functional.gelu(y)
    elif epi in (3, 4):
        ref = y + res.float()
    elif epi == 5:
        ur = res.float().requires_grad_(True)
        torch.nn.functional.gelu(ur).backward(y)
        ref = ur.grad
    else:
        ref = y
    tol = 1e-2 if odt == torch.bfloat16 else 1e-3
    assert (outs[0][0].float() - ref).abs().max().item() <= tol * ref.abs().max().item()


@pytest.mark.parametrize("b_is_nk", [True, False])
def test_pp_persistent_bert_shapes(gpu, b_is_nk):
    """The BERT-base layer shapes at C2 (M = 32768 rows) through the persistent form,
    B K-major (forward) and K-outer (the trainable encoder's dX): bit-identical to one
    workgroup per tile, several launches back to back on two streams (distinct tile
    counter slots)."""
    from irc_amd import ops

    g = torch.Generator().manual_seed(11)
    M, N, K = 32768, 3072, 768
    a = torch.randn(M, K, generator=g).bfloat16().to(gpu)
    b = (torch.randn(N, K, generator=g) if b_is_nk else torch.randn(K, N, generator=g))
    b = b.bfloat16().to(gpu)
    bias = torch.randn(N, generator=g).to(gpu)
    prev = ops.gemm_set_persistent(False)
    try:
        ref = ops.gemm(a, b, b_is_nk=b_is_nk, bias=bias, epilogue=2)
        torch.cuda.synchronize()
        ops.gemm_set_persistent(True)
        s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
        outs = []
        for st in (s1, s2, s1, s2):
            st.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(st):
                outs.append(ops.gemm(a, b, b_is_nk=b_is_nk, bias=bias, epilogue=2))
        torch.cuda.synchronize()
    finally:
        ops.gemm_set_persistent(prev)
    for o in outs:
        assert torch.equal(o, ref)
