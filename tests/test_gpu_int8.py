"""GPU parity of the int8 weight-only and int8 dynamic-activation paths against the oracle."""

import pytest
import torch

import torchao  # noqa: F401  (registers torch.ops.torchao)
from conftest import bf16, golden_files, golden_ms, load_golden
from oracle import oracle

pytestmark = pytest.mark.gpu
DEV = "cuda"
TOL_REF = 1e-2


@pytest.mark.parametrize("fname", golden_files("int8wo_"))
def test_int8wo_vs_reference_fixtures(fname):
    rec = load_golden(fname)
    q = torch.from_numpy(rec["q"])
    s, bias = bf16(rec["s"]), bf16(rec["bias"])
    for M in golden_ms(rec):
        x = bf16(rec[f"x_M{M}"])
        y = torch.ops.torchao.int8_weight_only_linear(
            x.to(DEV), q.to(DEV), s.to(DEV), bias.to(DEV)
        ).cpu()
        assert oracle.rel_l2(y, bf16(rec[f"y_M{M}"])) < TOL_REF


@pytest.mark.parametrize("M", [1, 2, 3, 4, 6, 8, 9, 16, 40, 128])
def test_int8wo_all_m_paths(M):
    N, K = 320, 2048
    w = oracle.make_linear_weight(N, K, seed=M)
    s = oracle.int8_weight_qparams(w)
    q = oracle.int8_weight_quantize(w, s)
    x = oracle.make_activation(M, K, seed=M + 1)
    y = torch.ops.torchao.int8_weight_only_linear(x.to(DEV), q.to(DEV), s.to(DEV), None).cpu()
    ref = oracle.int8wo_linear(x, q, s)
    assert oracle.rel_l2(y, ref) < TOL_REF
    exact = (x.double() @ q.double().t()) * s.double()
    assert oracle.rel_l2(y, exact) < 4e-3


@pytest.mark.parametrize("M,K", [(1, 4096), (7, 1024), (128, 4096), (33, 14336), (64, 16),
                                 (130, 8192), (3, 2064), (5, 8208)])
def test_int8_act_quant_bit_exact(M, K):
    x = oracle.make_activation(M, K, seed=K + M) * 3
    x[0] = 0.0
    if M > 2:
        x[2, 1] = 1000.0
    q, s = torch.ops.torchao.int8_quantize_per_token(x.to(DEV))
    q_ref, s_ref = oracle.int8_act_quant(x)
    assert torch.equal(s.cpu(), s_ref)
    assert torch.equal(q.cpu(), q_ref)


@pytest.mark.parametrize("M,K", [(128, 4096), (9, 2064), (4, 16)])
def test_int8_act_quant_wave_and_block_kernels_identical(M, K):
    """The one-wave-per-token kernel (token held in registers, the default for K <= 8192) and
    the 256-thread block kernel give the same bits."""
    from torchao.kernel import tuning

    x = (oracle.make_activation(M, K, seed=M * 7 + K) * 5).to(DEV)
    q0, s0 = torch.ops.torchao.int8_quantize_per_token(x)
    with tuning(int8_quant=1):
        q1, s1 = torch.ops.torchao.int8_quantize_per_token(x)
    assert torch.equal(q0, q1) and torch.equal(s0, s1)


@pytest.mark.parametrize("fname", golden_files("int8dyn_"))
def test_int8dyn_vs_reference_fixtures(fname):
    rec = load_golden(fname)
    wq = torch.from_numpy(rec["wq"])
    ws, bias = bf16(rec["ws"]), bf16(rec["bias"])
    for M in golden_ms(rec):
        x = bf16(rec[f"x_M{M}"])
        q, s = torch.ops.torchao.int8_quantize_per_token(x.to(DEV))
        assert torch.equal(q.cpu(), torch.from_numpy(rec[f"xq_M{M}"]))
        assert torch.equal(s.cpu().reshape(-1), bf16(rec[f"xs_M{M}"]))
        y = torch.ops.torchao.int8_scaled_mm(q, s, wq.to(DEV), ws.to(DEV), bias.to(DEV)).cpu()
        assert oracle.rel_l2(y, bf16(rec[f"y_M{M}"])) < TOL_REF
        # exact integer products + the reference epilogue order: bit exact to the reference
        assert torch.equal(y, bf16(rec[f"y_M{M}"]))


def test_int8_empty_and_batched_shapes():
    """Zero rows and leading batch dims, as torch.nn.functional.linear takes them: the int8
    weight-only op, the per-token quant and the int8 x int8 op keep the batch shape and give
    what the oracle gives row by row (zero rows launch nothing)."""
    N, K = 96, 512
    w = oracle.make_linear_weight(N, K, seed=5)
    s8 = oracle.int8_weight_qparams(w)
    q8 = oracle.int8_weight_quantize(w, s8)
    wq, ws = oracle.int8_dyn_weight(w)
    bias = oracle.make_activation(1, N, seed=6).reshape(N)
    x0 = torch.empty(0, K, dtype=torch.bfloat16, device=DEV)
    assert torch.ops.torchao.int8_weight_only_linear(x0, q8.to(DEV), s8.to(DEV), None).shape == (0, N)
    q0, s0 = torch.ops.torchao.int8_quantize_per_token(x0)
    assert q0.shape == (0, K) and s0.shape == (0, 1)
    assert torch.ops.torchao.int8_scaled_mm(q0, s0, wq.to(DEV), ws.to(DEV), None).shape == (0, N)

    x = oracle.make_activation(6, K, seed=8)
    xd = x.reshape(2, 3, K).to(DEV)
    y = torch.ops.torchao.int8_weight_only_linear(xd, q8.to(DEV), s8.to(DEV), bias.to(DEV))
    assert y.shape == (2, 3, N)
    assert oracle.rel_l2(y.cpu().reshape(6, N), oracle.int8wo_linear(x, q8, s8, bias)) < TOL_REF
    q, s = torch.ops.torchao.int8_quantize_per_token(xd)
    assert q.shape == (2, 3, K) and s.shape == (2, 3, 1)
    q_ref, s_ref = oracle.int8_act_quant(x)
    assert torch.equal(q.cpu().reshape(6, K), q_ref) and torch.equal(s.cpu().reshape(6, 1), s_ref)
    yd = torch.ops.torchao.int8_scaled_mm(q, s, wq.to(DEV), ws.to(DEV), bias.to(DEV))
    assert yd.shape == (2, 3, N)
    ref = oracle.int8_scaled_mm(q_ref, s_ref, wq, ws, bias, epilogue="cpu")
    assert torch.equal(yd.cpu().reshape(6, N), ref)


@pytest.mark.parametrize("M,N,K", [(128, 4096, 4096), (16, 512, 1024), (200, 320, 2048), (1, 256, 256)])
def test_int8_scaled_mm_exact_epilogue(M, N, K):
    w = oracle.make_linear_weight(N, K, seed=N)
    wq, ws = oracle.int8_dyn_weight(w)
    x = oracle.make_activation(M, K, seed=M)
    xq, xs = oracle.int8_act_quant(x)
    y = torch.ops.torchao.int8_scaled_mm(xq.to(DEV), xs.to(DEV), wq.to(DEV), ws.to(DEV), None).cpu()
    assert torch.equal(y, oracle.int8_scaled_mm(xq, xs, wq, ws, None, epilogue="cpu"))
    assert oracle.rel_l2(y, oracle.int8_scaled_mm(xq, xs, wq, ws, None, epilogue="fp32")) < TOL_REF


def test_int8_configs_end_to_end():
    from torchao.quantization import (
        Int8DynamicActivationInt8WeightConfig,
        Int8WeightOnlyConfig,
        quantize_,
    )

    K, N = 1024, 256
    base = torch.nn.Linear(K, N).to(torch.bfloat16)
    x = oracle.make_activation(64, K, seed=1)
    for cfg in (Int8WeightOnlyConfig(), Int8DynamicActivationInt8WeightConfig()):
        m = torch.nn.Linear(K, N).to(torch.bfloat16)
        m.load_state_dict(base.state_dict())
        m = m.to(DEV)
        quantize_(m, cfg)
        y = m(x.to(DEV)).cpu()
        ref = torch.nn.functional.linear(x.float(), base.weight.float(), base.bias.float())
        # quantization error dominates here: SQNR bar of the reference integration tests
        # (test_integration.py:978-1004 use >= 40 dB for int8wo; dynamic int8 is looser)
        sqnr = 20 * torch.log10(ref.norm() / (ref - y.float()).norm())
        assert sqnr > (35 if isinstance(cfg, Int8WeightOnlyConfig) else 25), (cfg, float(sqnr))


# ---- int8 x int8 decode GEMV (M <= 4) and the fused one-token linear -------------------------
# Integer products are exact and the epilogue is the reference's op order, so every check below
# is bit-exact (torch.equal) against the CPU oracle (oracle.int8_scaled_mm, epilogue "cpu").
DYN_SHAPES = [(256, 256), (40, 352), (4096, 4096), (6144, 4096), (4096, 14336), (1000, 11008),
              (128256 // 8, 4096)]


@pytest.mark.parametrize("M", [1, 2, 3, 4])
@pytest.mark.parametrize("N,K", DYN_SHAPES)
def test_int8dyn_gemv_bit_exact(M, N, K):
    w = oracle.make_linear_weight(N, K, seed=N + K)
    wq, ws = oracle.int8_dyn_weight(w)
    x = oracle.make_activation(M, K, seed=M + K) * 2
    if M > 1:
        x[1] = 0.0           # all-zero token: scale clamps to eps
    x[0, K // 3] = 500.0     # outlier
    xq, xs = oracle.int8_act_quant(x)
    bias = oracle.make_activation(1, N, seed=5).reshape(-1)
    for b in (None, bias):
        y = torch.ops.torchao.int8_scaled_mm(
            xq.to(DEV), xs.to(DEV), wq.to(DEV), ws.to(DEV), None if b is None else b.to(DEV)
        ).cpu()
        assert torch.equal(y, oracle.int8_scaled_mm(xq, xs, wq, ws, b, epilogue="cpu"))


@pytest.mark.parametrize("N,K", DYN_SHAPES + [(28672, 4096), (4096, 28672)])
def test_int8_dyn_linear_fused_bit_exact(N, K):
    w = oracle.make_linear_weight(N, K, seed=N)
    wq, ws = oracle.int8_dyn_weight(w)
    bias = oracle.make_activation(1, N, seed=9).reshape(-1)
    for seed, scale in ((1, 1.0), (2, 1e3), (3, 0.0)):
        x = oracle.make_activation(1, K, seed=seed) * scale
        xq, xs = oracle.int8_act_quant(x)
        for b in (None, bias):
            y = torch.ops.torchao.int8_dyn_linear(
                x.to(DEV), wq.to(DEV), ws.to(DEV), None if b is None else b.to(DEV)
            ).cpu()
            assert torch.equal(y, oracle.int8_scaled_mm(xq, xs, wq, ws, b, epilogue="cpu"))


def test_int8_dyn_gemv_launch_shapes_identical():
    """Every launch shape of the decode GEMV gives the same bits (exact integer sums)."""
    from torchao import _lib

    N, K = 1000, 11008
    w = oracle.make_linear_weight(N, K, seed=3)
    wq, ws = (t.to(DEV) for t in oracle.int8_dyn_weight(w))
    x = oracle.make_activation(1, K, seed=4).to(DEV)
    ref = torch.ops.torchao.int8_dyn_linear(x, wq, ws, None)
    try:
        for rpw in (2, 4, 8):
            for wk, g in ((1, 1), (2, 4), (4, 2), (8, 1), (3, 2)):
                _lib.call("tao_tune_int8_gemv", rpw, wk, g)
                assert torch.equal(torch.ops.torchao.int8_dyn_linear(x, wq, ws, None), ref)
                q, s = torch.ops.torchao.int8_quantize_per_token(x)
                assert torch.equal(torch.ops.torchao.int8_scaled_mm(q, s, wq, ws, None), ref)
    finally:
        _lib.call("tao_tune_int8_gemv", 0, 0, 0)


def test_int8_dyn_linear_args_fail_loudly():
    w = torch.zeros(64, 256, dtype=torch.int8, device=DEV)
    s = torch.ones(64, dtype=torch.bfloat16, device=DEV)
    with pytest.raises(RuntimeError):
        torch.ops.torchao.int8_dyn_linear(torch.zeros(2, 256, dtype=torch.bfloat16, device=DEV),
                                          w, s, None)
    with pytest.raises(RuntimeError):
        torch.ops.torchao.int8_dyn_linear(torch.zeros(1, 128, dtype=torch.bfloat16, device=DEV),
                                          w, s, None)


def test_int8dq_decode_takes_fused_path_and_matches_unfused():
    """quantize_(Int8DynamicActivationInt8WeightConfig) + one token on the GPU: the LAQT fast
    path (one launch) equals quantise -> F.linear(AQT x, AQT w), bit for bit, and the
    prefill-shaped input still takes the reference route."""
    from torchao.quantization import Int8DynamicActivationInt8WeightConfig, quantize_
    from torchao.quantization.linear_activation_quantized_tensor import _fused_int8_dyn_decode

    K, N = 4096, 1024
    m = torch.nn.Linear(K, N, bias=True).to(torch.bfloat16).to(DEV)
    quantize_(m, Int8DynamicActivationInt8WeightConfig())
    wt = m.weight
    for shape in ((1, K), (1, 1, K)):
        x = torch.randn(*shape, dtype=torch.bfloat16, device=DEV)
        assert _fused_int8_dyn_decode(x, wt, m.bias) is not None
        y = m(x)
        qx = wt.input_quant_func(x, **wt.quant_kwargs)
        y_ref = torch.nn.functional.linear(qx, wt.original_weight_tensor, m.bias)
        assert y.shape == y_ref.shape
        assert torch.equal(y, y_ref)
    assert _fused_int8_dyn_decode(torch.randn(4, K, dtype=torch.bfloat16, device=DEV), wt,
                                  None) is None


# ---- int8-dyn GEMM at M >= 48: the LDS-staged kernel (gemm_i8_lds_kernel) --------------------
# Forced on (tao_tune_gemm_algo 2) across ragged M / N, both M tiles and several K splits, with
# and without bias: bit-exact against the CPU oracle, and identical to the per-wave-column
# kernel (algo 1) on the same inputs.
@pytest.mark.parametrize("M,N,K", [(128, 4096, 4096), (48, 330, 1024), (200, 4160, 2048),
                                   (128, 14336, 4096), (128, 4096, 14336), (5, 64, 128),
                                   (512, 1024, 3072), (256, 4096, 4096), (128, 6144, 4096),
                                   (512, 14336, 4096), (300, 4200, 1024)])
def test_int8_lds_gemm_bit_exact(M, N, K):
    from torchao import _lib

    w = oracle.make_linear_weight(N, K, seed=N + 7)
    wq, ws = oracle.int8_dyn_weight(w)
    x = oracle.make_activation(M, K, seed=M + 3) * 2
    x[0, K // 5] = 300.0
    xq, xs = oracle.int8_act_quant(x)
    bias = oracle.make_activation(1, N, seed=9).reshape(-1)
    args = [t.to(DEV) for t in (xq, xs, wq, ws)]
    try:
        for b in (None, bias):
            ref = oracle.int8_scaled_mm(xq, xs, wq, ws, b, epilogue="cpu")
            bd = None if b is None else b.to(DEV)
            _lib.call("tao_tune_gemm_algo", 1)
            _lib.call("tao_tune_linear_crossover", 1)
            old = torch.ops.torchao.int8_scaled_mm(*args, bd).cpu()
            _lib.call("tao_tune_gemm_algo", 2)
            for bm, splits, depth in ((0, 0, 0), (64, 1, 0), (128, 1, 0), (64, 3, 0),
                                      (128, 8, 0), (64, 1, 2), (64, 2, 8), (128, 1, 6),
                                      (128, 3, 2)):
                for bn in ((64, 128) if depth in (0, 2) else (64,)):
                    _lib.call("tao_tune_gemm", bm, 0, splits)
                    _lib.call("tao_tune_gemm_depth", depth)
                    _lib.call("tao_tune_gemm_bn", bn)
                    y = torch.ops.torchao.int8_scaled_mm(*args, bd).cpu()
                    assert torch.equal(y, ref), (bm, splits, depth, bn)
            _lib.call("tao_tune_gemm_depth", 0)
            _lib.call("tao_tune_gemm_bn", 0)
            assert torch.equal(old, ref)
            _lib.call("tao_tune_gemm", 0, 0, 0)
            _lib.call("tao_tune_gemm_algo", 0)  # the auto policy's pick for this shape
            assert torch.equal(torch.ops.torchao.int8_scaled_mm(*args, bd).cpu(), ref)
    finally:
        _lib.call("tao_tune_gemm", 0, 0, 0)
        _lib.call("tao_tune_gemm_depth", 0)
        _lib.call("tao_tune_gemm_bn", 0)
        _lib.call("tao_tune_gemm_algo", 0)
        _lib.call("tao_tune_linear_crossover", 0)


# ---- torchao.kernel.intmm (reference kernel/intmm.py:30-143), VERDICT r2 W6 --------------------
@pytest.mark.parametrize("M", [1, 8, 16, 17, 128])
@pytest.mark.parametrize("b_layout", ["weight_t", "contiguous"])
def test_int_scaled_matmul_bit_exact(M, b_layout):
    """int_scaled_matmul(a, b, s) == bf16(bf16(a @ b) * s), the reference's epilogue on both
    devices, bit for bit: b = w.t() of a contiguous [N, K] weight takes the fused int8-MFMA/GEMV
    kernel; a contiguous [K, N] b takes safe_int_mm (hipBLASLt or the exact fp64 fallback) then the
    torch multiply."""
    from torchao.kernel.intmm import int_scaled_matmul

    N, K = 256, 1024
    w = oracle.make_linear_weight(N, K, seed=M)
    wq, _ = oracle.int8_dyn_weight(w)
    x = oracle.make_activation(M, K, seed=M + 3)
    xq, xs = oracle.int8_act_quant(x)
    b = wq.t().to(DEV) if b_layout == "weight_t" else wq.t().contiguous().to(DEV)
    y = int_scaled_matmul(xq.to(DEV), b, xs.to(DEV)).cpu()
    ref = oracle.int8_scaled_mm(xq, xs, wq, torch.ones(N, dtype=torch.bfloat16))
    assert y.dtype == torch.bfloat16 and torch.equal(y, ref)


@pytest.mark.parametrize("M,K,N", [(1, 4096, 4096), (8, 1024, 256), (16, 1024, 256),
                                   (17, 1024, 256), (128, 4096, 4096), (5, 1000, 36)])
def test_safe_int_mm_exact(M, K, N):
    """safe_int_mm is exact int32 at every M (no int32 torch.mm on the device, which PyTorch has no
    kernel for), including full-range operands whose sums exceed fp32's exact range, and shapes
    the BLAS path rejects (K, N not multiples of 8: the reference's host fallback)."""
    from torchao.kernel.intmm import safe_int_mm

    g = torch.Generator().manual_seed(M * K + N)
    a = torch.randint(-128, 128, (M, K), generator=g, dtype=torch.int8)
    b = torch.randint(-128, 128, (K, N), generator=g, dtype=torch.int8)
    a[0, :] = -128
    b[:, 0] = -128  # y[0, 0] = K * 2^14 > 2^24 at K = 4096
    c = safe_int_mm(a.to(DEV), b.to(DEV))
    assert c.dtype == torch.int32 and c.device.type == "cuda"
    exact = (a.to(torch.int64) @ b.to(torch.int64)).to(torch.int32)
    assert torch.equal(c.cpu(), exact)


def test_intmm_mixed_devices_raise():
    from torchao.kernel.intmm import int_scaled_matmul, safe_int_mm

    a = torch.zeros(4, 64, dtype=torch.int8, device=DEV)
    b = torch.zeros(64, 32, dtype=torch.int8)
    with pytest.raises(AssertionError, match="same device"):
        safe_int_mm(a, b)
    with pytest.raises(AssertionError, match="same device"):
        int_scaled_matmul(a, b, torch.ones(4, 1, dtype=torch.bfloat16, device=DEV))
