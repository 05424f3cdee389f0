"""GPU parity of the weight-shared tile GEMM (csrc/gemm_tile.hip) against the CPU oracle.

The kernel serves the quantized linears at M >= 64 (prefill): 4 waves split the rows of a
64/128 x 64 tile, each step's weights are dequantised once per workgroup into LDS, x fragments
come straight from global memory, and K is split S ways with every slice reducing 1/S of the tile.
Checked here: every path (int4 all group sizes, int8 weight-only, int8 dynamic bit-exact) over
both row tiles, partial M and N tiles, forced splits 1..16 (including more slices than steps),
bias, run-to-run bit identity, graph capture, and that a captured graph's split-K workspace is
released with the graph.
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
def tile():
    yield lambda mode, splits=0: _lib.call("tao_tune_gemm_tile", mode, splits)
    _lib.call("tao_tune_gemm_tile", 0, 0)


def _int4(N, K, g, seed):
    w = oracle.make_linear_weight(N, K, seed=seed)
    s, z = oracle.int4_qparams(w, g)
    q = oracle.int4_quantize(w, s, z, g)
    packed = torch.ops.torchao.int4_pack(q.to(DEV))
    sz = torch.stack([s, z], dim=-1).contiguous().to(DEV)
    return q, s, z, packed, sz


SHAPES = [(64, 4096, 1024), (65, 200, 512), (128, 4096, 4096), (200, 1000, 2048),
          (256, 4096, 1024), (97, 64, 256), (300, 6144, 4096)]


@pytest.mark.parametrize("M,N,K", SHAPES)
@pytest.mark.parametrize("g", [32, 128])
def test_tile_int4(tile, M, N, K, g):
    tile(2)
    q, s, z, packed, sz = _int4(N, K, g, seed=M + N + g)
    x = oracle.make_activation(M, K, seed=M)
    bias = oracle.make_activation(1, N, seed=7).reshape(N)
    y = torch.ops.torchao.int4_weight_only_linear(x.to(DEV), packed, sz, g, bias.to(DEV)).cpu()
    assert oracle.rel_l2(y, oracle.int4_linear(x, q, s, z, g, bias)) < TOL_REF
    assert oracle.rel_l2(y, oracle.int4_linear_fp32(x, q, s, z, g, bias)) < TOL_FP32


@pytest.mark.parametrize("g", [64, 256])
def test_tile_int4_group_sizes(tile, g):
    tile(2)
    M, N, K = 128, 512, 2048
    q, s, z, packed, sz = _int4(N, K, g, seed=g)
    x = oracle.make_activation(M, K, seed=g)
    y = torch.ops.torchao.int4_weight_only_linear(x.to(DEV), packed, sz, g, None).cpu()
    assert oracle.rel_l2(y, oracle.int4_linear_fp32(x, q, s, z, g)) < TOL_FP32


@pytest.mark.parametrize("M,N,K", SHAPES)
def test_tile_int8wo(tile, M, N, K):
    tile(2)
    w = oracle.make_linear_weight(N, K, seed=M + N)
    s = oracle.int8_weight_qparams(w)
    q = oracle.int8_weight_quantize(w, s)
    x = oracle.make_activation(M, K, seed=M)
    y = torch.ops.torchao.int8_weight_only_linear(x.to(DEV), q.to(DEV), s.to(DEV), None).cpu()
    assert oracle.rel_l2(y, oracle.int8wo_linear(x, q, s)) < TOL_REF
    exact = (x.double() @ q.double().t()) * s.double()
    assert oracle.rel_l2(y, exact) < TOL_FP32


@pytest.mark.parametrize("M,N,K", SHAPES + [(128, 4096, 14336), (512, 1024, 4096)])
def test_tile_int8dyn_bit_exact(tile, M, N, K):
    tile(2)
    w = oracle.make_linear_weight(N, K, seed=M + N)
    wq, ws = oracle.int8_dyn_weight(w)
    x = oracle.make_activation(M, K, seed=M)
    xq, xs = oracle.int8_act_quant(x)
    bias = oracle.make_activation(1, N, seed=3).reshape(N)
    y = torch.ops.torchao.int8_scaled_mm(
        xq.to(DEV), xs.to(DEV), wq.to(DEV), ws.to(DEV), bias.to(DEV)).cpu()
    assert torch.equal(y, oracle.int8_scaled_mm(xq, xs, wq, ws, bias, epilogue="cpu"))


@pytest.mark.parametrize("splits", [1, 2, 4, 8, 16, 64])
def test_tile_forced_splits(tile, splits):
    """Every split count (64 clamps to 16; 16 slices of a 1024-k int8 weight = more than its 4
    steps allow, clamped to 2 steps per slice), back to back so the epoch counters advance."""
    M, N, K = 128, 256, 2048
    w = oracle.make_linear_weight(N, K, seed=splits)
    wq, ws = oracle.int8_dyn_weight(w)
    x = oracle.make_activation(M, K, seed=splits)
    xq, xs = oracle.int8_act_quant(x)
    ref = oracle.int8_scaled_mm(xq, xs, wq, ws, None, epilogue="cpu")
    q, s, z, packed, sz = _int4(N, K, 32, seed=splits)
    ref4 = oracle.int4_linear_fp32(x, q, s, z, 32)
    tile(2, splits)
    for _ in range(3):
        y = torch.ops.torchao.int8_scaled_mm(xq.to(DEV), xs.to(DEV), wq.to(DEV), ws.to(DEV), None)
        assert torch.equal(y.cpu(), ref)
        y4 = torch.ops.torchao.int4_weight_only_linear(x.to(DEV), packed, sz, 32, None).cpu()
        assert oracle.rel_l2(y4, ref4) < TOL_FP32


def test_tile_deterministic_and_matches_old_kernel(tile):
    """Run-to-run bit identity (fixed slab-sum order), and agreement with gemm_mfma.hip's
    kernel (bit-identical for int8 dyn; one fp32 summation order apart for int4)."""
    M, N, K, g = 128, 4096, 4096, 32
    q, s, z, packed, sz = _int4(N, K, g, seed=1)
    x = oracle.make_activation(M, K, seed=2).to(DEV)
    tile(2)
    a = torch.ops.torchao.int4_weight_only_linear(x, packed, sz, g, None)
    for _ in range(3):
        assert torch.equal(torch.ops.torchao.int4_weight_only_linear(x, packed, sz, g, None), a)
    tile(1)
    old = torch.ops.torchao.int4_weight_only_linear(x, packed, sz, g, None)
    assert oracle.rel_l2(a.cpu(), old.cpu()) < 2e-3
    w = oracle.make_linear_weight(N, K, seed=3)
    wq, ws = oracle.int8_dyn_weight(w)
    xq, xs = oracle.int8_act_quant(x.cpu())
    args = (xq.to(DEV), xs.to(DEV), wq.to(DEV), ws.to(DEV), None)
    old8 = torch.ops.torchao.int8_scaled_mm(*args)
    tile(2)
    assert torch.equal(torch.ops.torchao.int8_scaled_mm(*args), old8)


def test_tile_graph_capture_and_workspace_released(tile):
    """Replays equal eager; re-capturing and destroying graphs with split-K launches does not
    accumulate workspaces or device memory (each is owned by its graph)."""
    tile(2, 4)
    M, N, K, g = 128, 1024, 2048, 32
    q, s, z, packed, sz = _int4(N, K, g, seed=4)
    x = oracle.make_activation(M, K, seed=5).to(DEV)
    eager = torch.ops.torchao.int4_weight_only_linear(x, packed, sz, g, None)
    stream = torch.cuda.Stream()
    torch.cuda.synchronize()
    base = _lib.lib().tao_graph_workspace_count()
    free0 = None
    for it in range(6):
        graph = torch.cuda.CUDAGraph()
        stream.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(stream):
            with torch.cuda.graph(graph, stream=stream):
                out = torch.ops.torchao.int4_weight_only_linear(x, packed, sz, g, None)
        torch.cuda.current_stream().wait_stream(stream)
        assert _lib.lib().tao_graph_workspace_count() == base + 1
        # an eager split-K launch needing a larger workspace between capture and
        # replay (the step that frees retired buffers) must not free the graph's one
        xb = oracle.make_activation(256, K, seed=6).to(DEV)
        big = torch.ops.torchao.int4_weight_only_linear(xb, packed, sz, g, None)
        torch.cuda.synchronize()
        assert _lib.lib().tao_graph_workspace_count() == base + 1
        assert big.shape == (256, N)
        del xb, big
        for _ in range(2):
            graph.replay()
        torch.cuda.synchronize()
        assert torch.equal(out, eager)
        del graph, out
        torch.cuda.synchronize()
        # the user-object destructor may run asynchronously; the next eager split-K call frees
        # what destroyed graphs left
        import time

        t0 = time.time()
        while _lib.lib().tao_graph_workspace_count() != base and time.time() - t0 < 2.0:
            time.sleep(0.01)
        assert _lib.lib().tao_graph_workspace_count() == base
        torch.ops.torchao.int4_weight_only_linear(x, packed, sz, g, None)
        torch.cuda.synchronize()
        free = torch.cuda.mem_get_info()[0]
        if it == 1:
            free0 = free
        elif it > 1:
            assert free >= free0 - (8 << 20), (free0, free)
