"""GPU parity of the k-split prefill GEMM (csrc/gemm_ksplit.hip) against the CPU oracle.

One 32 x 64 output tile per workgroup over the whole K; the workgroup's 8 (or 16) waves split K
between them (wave w takes k-blocks w, w + NW, ...), load their operands straight into MFMA
fragments, and sum their partial tiles through LDS in wave order. Checked here, through the C-ABI
(torch.ops.torchao.*): int4 at every group size against the reference dequant -> F.linear bar and
the fp32 accumulation of the same weights; int8 dynamic BIT-EXACT against the reference CPU
epilogue (int32 sums are exact in any order); every launch shape (waves, ring depth, and the
depth halved until it divides the wave's blocks); partial M tiles (rows clamped on load, masked
on store); long K; saturated int8 operands; bias; run-to-run bit identity; agreement with
gemm_mfma.hip's kernels; graph capture; and that unsupported shapes fall back.
"""

import pytest
import torch

from oracle import oracle

from torchao import _lib

pytestmark = pytest.mark.gpu
DEV = "cuda"
TOL_REF = 1e-2
TOL_FP32 = 4e-3


@pytest.fixture
def ksplit():
    yield lambda mode, shape=0: _lib.call("tao_tune_gemm_ksplit", mode, shape)
    _lib.call("tao_tune_reset")


def _int4(N, K, g, seed):
    w = oracle.make_linear_weight(N, K, seed=seed)
    s, z = oracle.int4_qparams(w, g)
    q = oracle.int4_quantize(w, s, z, g)
    packed = torch.ops.torchao.int4_pack(q.to(DEV))
    sz = torch.stack([s, z], dim=-1).contiguous().to(DEV)
    return q, s, z, packed, sz


# (M, N, K): full and partial 32-row tiles; K = 1024 (one block per wave) up to 14336; K = 3072
# (3 blocks per wave: the ring depth drops to 1)
INT4_SHAPES = [(128, 4096, 4096), (5, 64, 1024), (17, 128, 1024), (33, 192, 2048), (64, 256, 2048),
               (100, 640, 4096), (256, 1024, 3072), (128, 512, 14336), (300, 128, 2048)]


@pytest.mark.parametrize("M,N,K", INT4_SHAPES)
@pytest.mark.parametrize("g", [32, 128])
@pytest.mark.parametrize("shape", [0, 1, 3, 4, 17])
def test_ksplit_int4(ksplit, M, N, K, g, shape):
    """Every output tile (32 x 64, 64 x 32, 128 x 16), ring depth and the rotated block order."""
    ksplit(2, shape)
    q, s, z, packed, sz = _int4(N, K, g, seed=M + N + g)
    x = oracle.make_activation(M, K, seed=M)
    bias = oracle.make_activation(1, N, seed=7).reshape(N)
    y = torch.ops.torchao.int4_weight_only_linear(x.to(DEV), packed, sz, g, bias.to(DEV)).cpu()
    assert y.shape == (M, N)
    assert oracle.rel_l2(y, oracle.int4_linear(x, q, s, z, g, bias)) < TOL_REF
    assert oracle.rel_l2(y, oracle.int4_linear_fp32(x, q, s, z, g, bias)) < TOL_FP32


@pytest.mark.parametrize("g", [64, 256])
@pytest.mark.parametrize("shape", [1, 3])
def test_ksplit_int4_group_sizes_and_shapes(ksplit, g, shape):
    """g = 64 and 256: the (scale, zero) word index (4 kb + q) >> log2(g / 32) splits into a block
    part and a lane part; two output tiles."""
    ksplit(2, shape)
    M, N, K = 96, 320, 6144
    q, s, z, packed, sz = _int4(N, K, g, seed=g)
    x = oracle.make_activation(M, K, seed=g)
    y = torch.ops.torchao.int4_weight_only_linear(x.to(DEV), packed, sz, g, None).cpu()
    assert oracle.rel_l2(y, oracle.int4_linear_fp32(x, q, s, z, g)) < TOL_FP32
    assert oracle.rel_l2(y, oracle.int4_linear(x, q, s, z, g)) < TOL_REF


INT8_SHAPES = [(128, 4096, 4096), (5, 64, 512), (31, 128, 1024), (33, 192, 2048),
               (64, 4096, 3072), (128, 512, 14336), (256, 1024, 4096), (300, 256, 1536)]


@pytest.mark.parametrize("M,N,K", INT8_SHAPES)
@pytest.mark.parametrize("shape", [0, 1, 2, 3, 4, 17, 19])
def test_ksplit_int8dyn_bit_exact(ksplit, M, N, K, shape):
    ksplit(2, shape)
    w = oracle.make_linear_weight(N, K, seed=M + N)
    wq, ws = oracle.int8_dyn_weight(w)
    x = oracle.make_activation(M, K, seed=M)
    xq, xs = oracle.int8_act_quant(x)
    bias = oracle.make_activation(1, N, seed=3).reshape(N)
    y = torch.ops.torchao.int8_scaled_mm(
        xq.to(DEV), xs.to(DEV), wq.to(DEV), ws.to(DEV), bias.to(DEV)).cpu()
    assert torch.equal(y, oracle.int8_scaled_mm(xq, xs, wq, ws, bias, epilogue="cpu"))
    y = torch.ops.torchao.int8_scaled_mm(xq.to(DEV), xs.to(DEV), wq.to(DEV), ws.to(DEV), None).cpu()
    assert torch.equal(y, oracle.int8_scaled_mm(xq, xs, wq, ws, None, epilogue="cpu"))


def test_ksplit_int8dyn_extreme_values(ksplit):
    """Saturated int8 operands (+-127 everywhere, long K): the int32 sums reach 127^2 K and stay
    exact through the i8 MFMAs and the cross-wave sum."""
    ksplit(2)
    M, N, K = 64, 128, 8192
    g = torch.Generator().manual_seed(0)
    wq = (torch.randint(0, 2, (N, K), generator=g, dtype=torch.int8) * 254 - 127).to(torch.int8)
    xq = (torch.randint(0, 2, (M, K), generator=g, dtype=torch.int8) * 254 - 127).to(torch.int8)
    ws = torch.full((N,), 1e-4).to(torch.bfloat16)
    xs = torch.full((M,), 1e-3).to(torch.bfloat16)
    y = torch.ops.torchao.int8_scaled_mm(xq.to(DEV), xs.to(DEV), wq.to(DEV), ws.to(DEV), None).cpu()
    assert torch.equal(y, oracle.int8_scaled_mm(xq, xs, wq, ws, None, epilogue="cpu"))


def test_ksplit_deterministic_and_matches_old_kernel(ksplit):
    """Run-to-run bit identity, and agreement with gemm_mfma.hip's kernels (bit-identical for
    int8 dyn; fp32 summation orders apart for int4)."""
    M, N, K, g = 128, 4096, 4096, 32
    q, s, z, packed, sz = _int4(N, K, g, seed=1)
    x = oracle.make_activation(M, K, seed=2).to(DEV)
    ksplit(2)
    a = torch.ops.torchao.int4_weight_only_linear(x, packed, sz, g, None)
    for _ in range(3):
        assert torch.equal(torch.ops.torchao.int4_weight_only_linear(x, packed, sz, g, None), a)
    ksplit(1)
    old = torch.ops.torchao.int4_weight_only_linear(x, packed, sz, g, None)
    assert oracle.rel_l2(a.cpu(), old.cpu()) < 2e-3
    w = oracle.make_linear_weight(N, K, seed=3)
    wq, ws = oracle.int8_dyn_weight(w)
    xq, xs = oracle.int8_act_quant(x.cpu())
    args = (xq.to(DEV), xs.to(DEV), wq.to(DEV), ws.to(DEV), None)
    old8 = torch.ops.torchao.int8_scaled_mm(*args)
    ksplit(2)
    assert torch.equal(torch.ops.torchao.int8_scaled_mm(*args), old8)


def test_ksplit_graph_capture(ksplit):
    ksplit(2)
    M, N, K, g = 128, 1024, 2048, 32
    q, s, z, packed, sz = _int4(N, K, g, seed=4)
    x = oracle.make_activation(M, K, seed=5).to(DEV)
    eager = torch.ops.torchao.int4_weight_only_linear(x, packed, sz, g, None)
    side = torch.cuda.Stream()
    graph = torch.cuda.CUDAGraph()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        with torch.cuda.graph(graph, stream=side):
            out = torch.ops.torchao.int4_weight_only_linear(x, packed, sz, g, None)
    torch.cuda.current_stream().wait_stream(side)
    for _ in range(3):
        graph.replay()
    torch.cuda.synchronize()
    assert torch.equal(out, eager)


def test_ksplit_unsupported_shapes_fall_back(ksplit):
    """N not a multiple of 64 or K not a multiple of the waves' blocks: the forced mode still
    routes to the other kernels (results within the oracle bars)."""
    ksplit(2)
    for (M, N, K) in [(64, 200, 1024), (64, 256, 1056), (64, 256, 1536)]:
        q, s, z, packed, sz = _int4(N, K, 32, seed=N)
        x = oracle.make_activation(M, K, seed=K)
        y = torch.ops.torchao.int4_weight_only_linear(x.to(DEV), packed, sz, 32, None).cpu()
        assert oracle.rel_l2(y, oracle.int4_linear_fp32(x, q, s, z, 32)) < TOL_FP32
    M, N, K = 64, 256, 1056  # int8: K not a multiple of 512
    w = oracle.make_linear_weight(N, K, seed=9)
    wq, ws = oracle.int8_dyn_weight(w)
    x = oracle.make_activation(M, K, seed=9)
    xq, xs = oracle.int8_act_quant(x)
    y = torch.ops.torchao.int8_scaled_mm(xq.to(DEV), xs.to(DEV), wq.to(DEV), ws.to(DEV), None).cpu()
    assert torch.equal(y, oracle.int8_scaled_mm(xq, xs, wq, ws, None, epilogue="cpu"))
