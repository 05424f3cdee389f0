"""GPU parity of the MFMA skinny GEMM (gemm_mfma.hip) across its M tiles and edge shapes.

The kernel picks BM in {16, 32, 64, 128} from (M, N) so the grid covers the chip; the shapes
below force each tile, partial last M tiles, N not a multiple of the 64-column block, and K
that is not a multiple of the macro-step (128 bf16 k / 256 int8 k) or shorter than the
prefetch depth. The GEMV <-> MFMA crossover is moved with tao_tune_linear_crossover so M 5..8
is checked on both kernels.
"""

import pytest
import torch

from oracle import oracle

from torchao import _lib

pytestmark = pytest.mark.gpu
DEV = "cuda"
TOL_REF = 1e-2
TOL_FP32 = 4e-3

# (M, N, K): tile chosen by choose_bm in brackets
SHAPES = [
    (5, 4096, 1024),    # [16] smallest MFMA M
    (48, 4096, 1024),   # [16] 3 M tiles
    (129, 4096, 1024),  # [32] partial last tile
    (300, 4096, 1024),  # [64] partial last tile
    (600, 4096, 1024),  # [128] partial last tile
    (128, 200, 352),    # [16] ragged N, K not a multiple of the step
    (40, 72, 32),       # [16] single partial step, N tail of 8
]


@pytest.fixture
def crossover():
    yield lambda m: _lib.call("tao_tune_linear_crossover", m)
    _lib.call("tao_tune_linear_crossover", 0)


@pytest.fixture
def gemm_shape():
    yield lambda bm, kg, splits: _lib.call("tao_tune_gemm", bm, kg, splits)
    _lib.call("tao_tune_gemm", 0, 0, 0)


@pytest.mark.parametrize("M,N,K", SHAPES)
def test_int4_mfma_tiles(M, N, K):
    g = 32
    w = oracle.make_linear_weight(N, K, seed=M + N)
    s, z = oracle.int4_qparams(w, g)
    q = oracle.int4_quantize(w, s, z, g)
    x = oracle.make_activation(M, K, seed=M)
    bias = oracle.make_activation(1, N, seed=7).reshape(N)
    packed = torch.ops.torchao.int4_pack(q.to(DEV))
    sz = torch.stack([s, z], dim=-1).contiguous().to(DEV)
    y = torch.ops.torchao.int4_weight_only_linear(x.to(DEV), packed, sz, g, bias.to(DEV)).cpu()
    assert oracle.rel_l2(y, oracle.int4_linear(x, q, s, z, g, bias)) < TOL_REF
    assert oracle.rel_l2(y, oracle.int4_linear_fp32(x, q, s, z, g, bias)) < TOL_FP32


@pytest.mark.parametrize("M,N,K", SHAPES)
def test_int8wo_mfma_tiles(M, N, K):
    w = oracle.make_linear_weight(N, K, seed=M + N)
    s = oracle.int8_weight_qparams(w)
    q = oracle.int8_weight_quantize(w, s)
    x = oracle.make_activation(M, K, seed=M)
    y = torch.ops.torchao.int8_weight_only_linear(x.to(DEV), q.to(DEV), s.to(DEV), None).cpu()
    assert oracle.rel_l2(y, oracle.int8wo_linear(x, q, s)) < TOL_REF
    exact = (x.double() @ q.double().t()) * s.double()
    assert oracle.rel_l2(y, exact) < TOL_FP32


@pytest.mark.parametrize("M,N,K", SHAPES + [(512, 4096, 4096), (7, 64, 16)])
def test_int8dyn_mfma_tiles_bit_exact(M, N, K):
    w = oracle.make_linear_weight(N, K, seed=M + N)
    wq, ws = oracle.int8_dyn_weight(w)
    x = oracle.make_activation(M, K, seed=M)
    xq, xs = oracle.int8_act_quant(x)
    bias = oracle.make_activation(1, N, seed=3).reshape(N)
    y = torch.ops.torchao.int8_scaled_mm(
        xq.to(DEV), xs.to(DEV), wq.to(DEV), ws.to(DEV), bias.to(DEV)
    ).cpu()
    # integer accumulation is exact, the epilogue follows the reference's rounding order
    assert torch.equal(y, oracle.int8_scaled_mm(xq, xs, wq, ws, bias, epilogue="cpu"))


@pytest.mark.parametrize("M", [5, 6, 7, 8])
@pytest.mark.parametrize("max_gemv_m", [4, 8])
def test_crossover_both_kernels(crossover, M, max_gemv_m):
    crossover(max_gemv_m)
    N, K, g = 1024, 2048, 64
    w = oracle.make_linear_weight(N, K, seed=M)
    s, z = oracle.int4_qparams(w, g)
    q = oracle.int4_quantize(w, s, z, g)
    x = oracle.make_activation(M, K, seed=M + 9)
    packed = torch.ops.torchao.int4_pack(q.to(DEV))
    sz = torch.stack([s, z], dim=-1).contiguous().to(DEV)
    y = torch.ops.torchao.int4_weight_only_linear(x.to(DEV), packed, sz, g, None).cpu()
    assert oracle.rel_l2(y, oracle.int4_linear_fp32(x, q, s, z, g)) < TOL_FP32
    s8 = oracle.int8_weight_qparams(w)
    q8 = oracle.int8_weight_quantize(w, s8)
    y8 = torch.ops.torchao.int8_weight_only_linear(x.to(DEV), q8.to(DEV), s8.to(DEV), None).cpu()
    assert oracle.rel_l2(y8, oracle.int8wo_linear(x, q8, s8)) < TOL_REF


def test_crossover_rejects_out_of_range():
    with pytest.raises(RuntimeError, match="max_gemv_m"):
        _lib.call("tao_tune_linear_crossover", 9)


# forced (M tile, k-groups, K slices): every tile with and without both K splits, uneven
# slices and k-groups with idle steps (K=1056 has 9 int4 steps / 5 int8 steps), more slices
# than steps (clamped), the partial-sum protocol reused back to back (counters reset by the
# last arriver)
FORCED = [(16, 1, 1), (16, 4, 1), (16, 2, 3), (32, 4, 4), (32, 1, 2), (64, 2, 2), (64, 1, 1),
          (128, 1, 5), (16, 4, 64), (32, 2, 16)]


@pytest.mark.parametrize("bm,kg,splits", FORCED)
def test_forced_tiles_and_split_k(gemm_shape, bm, kg, splits):
    gemm_shape(bm, kg, splits)
    M, N, K, g = 70, 320, 1056, 32
    w = oracle.make_linear_weight(N, K, seed=bm + kg + splits)
    s, z = oracle.int4_qparams(w, g)
    q = oracle.int4_quantize(w, s, z, g)
    x = oracle.make_activation(M, K, seed=splits)
    bias = oracle.make_activation(1, N, seed=5).reshape(N)
    packed = torch.ops.torchao.int4_pack(q.to(DEV))
    sz = torch.stack([s, z], dim=-1).contiguous().to(DEV)
    xd, bd = x.to(DEV), bias.to(DEV)
    y = torch.ops.torchao.int4_weight_only_linear(xd, packed, sz, g, bd)
    y2 = torch.ops.torchao.int4_weight_only_linear(xd, packed, sz, g, bd)
    assert torch.equal(y, y2)  # slices are summed in a fixed order
    assert oracle.rel_l2(y.cpu(), oracle.int4_linear_fp32(x, q, s, z, g, bias)) < TOL_FP32

    s8 = oracle.int8_weight_qparams(w)
    q8 = oracle.int8_weight_quantize(w, s8)
    y8 = torch.ops.torchao.int8_weight_only_linear(xd, q8.to(DEV), s8.to(DEV), bd).cpu()
    assert oracle.rel_l2(y8, oracle.int8wo_linear(x, q8, s8, bias)) < TOL_REF

    wq, ws = oracle.int8_dyn_weight(w)
    xq, xs = oracle.int8_act_quant(x)
    yd = torch.ops.torchao.int8_scaled_mm(xq.to(DEV), xs.to(DEV), wq.to(DEV), ws.to(DEV), bd)
    assert torch.equal(yd.cpu(), oracle.int8_scaled_mm(xq, xs, wq, ws, bias, epilogue="cpu"))


def test_split_k_under_graph_capture(gemm_shape):
    """The workspace is reserved by the eager call; the captured launch reuses it."""
    gemm_shape(16, 4, 8)
    M, N, K, g = 16, 512, 2048, 32
    w = oracle.make_linear_weight(N, K, seed=3)
    s, z = oracle.int4_qparams(w, g)
    q = oracle.int4_quantize(w, s, z, g)
    x = oracle.make_activation(M, K, seed=4).to(DEV)
    packed = torch.ops.torchao.int4_pack(q.to(DEV))
    sz = torch.stack([s, z], dim=-1).contiguous().to(DEV)
    stream = torch.cuda.Stream()
    with torch.cuda.stream(stream):
        ref = torch.ops.torchao.int4_weight_only_linear(x, packed, sz, g, None)
        stream.synchronize()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=stream):
            out = torch.ops.torchao.int4_weight_only_linear(x, packed, sz, g, None)
    for _ in range(3):
        graph.replay()
    torch.cuda.synchronize()
    assert torch.equal(out, ref)


def test_tune_gemm_rejects_bad_values():
    with pytest.raises(RuntimeError, match="m_tile"):
        _lib.call("tao_tune_gemm", 48, 0, 0)
    with pytest.raises(RuntimeError, match="k_groups"):
        _lib.call("tao_tune_gemm", 0, 3, 0)
    with pytest.raises(RuntimeError, match="splits"):
        _lib.call("tao_tune_gemm", 0, 0, 65)


def _int4_operands(M, N, K, g, seed):
    w = oracle.make_linear_weight(N, K, seed=seed)
    s, z = oracle.int4_qparams(w, g)
    q = oracle.int4_quantize(w, s, z, g)
    x = oracle.make_activation(M, K, seed=seed + 1)
    packed = torch.ops.torchao.int4_pack(q.to(DEV))
    sz = torch.stack([s, z], dim=-1).contiguous().to(DEV)
    return x, q, s, z, packed, sz


def test_split_k_capture_owns_its_workspace():
    """a captured split-K launch must not share scratch with eager work.
    Capture at a small split-K shape, then run a LARGER split-K shape eagerly on the capture
    stream (which grows, and frees, that stream's eager workspace) and on another stream; every
    later replay must still reproduce the eager result exactly."""
    from torchao.kernel import tuning

    g = 32
    x1, q1, s1, z1, p1, sz1 = _int4_operands(16, 512, 2048, g, seed=11)
    x2, q2, s2, z2, p2, sz2 = _int4_operands(64, 4096, 8192, g, seed=12)
    x1, x2 = x1.to(DEV), x2.to(DEV)
    stream = torch.cuda.Stream()
    with tuning(gemm=(16, 1, 8)):
        with torch.cuda.stream(stream):
            ref1 = torch.ops.torchao.int4_weight_only_linear(x1, p1, sz1, g, None)
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph, stream=stream):
                out1 = torch.ops.torchao.int4_weight_only_linear(x1, p1, sz1, g, None)
            ref2 = torch.ops.torchao.int4_weight_only_linear(x2, p2, sz2, g, None)
        other = torch.cuda.Stream()
        with torch.cuda.stream(other):
            ref2b = torch.ops.torchao.int4_weight_only_linear(x2, p2, sz2, g, None)
        torch.cuda.synchronize()
        for _ in range(3):
            out1.zero_()
            graph.replay()
            torch.cuda.synchronize()
            assert torch.equal(out1, ref1)
        # replay concurrently with eager split-K work on another stream: disjoint scratch
        with torch.cuda.stream(other):
            again2 = torch.ops.torchao.int4_weight_only_linear(x2, p2, sz2, g, None)
        graph.replay()
        torch.cuda.synchronize()
        assert torch.equal(out1, ref1)
        assert torch.equal(again2, ref2b) and torch.equal(ref2, ref2b)
    y = ref2.cpu()
    assert oracle.rel_l2(y, oracle.int4_linear_fp32(x2.cpu(), q2, s2, z2, g)) < TOL_FP32


@pytest.mark.parametrize("fmt", ["int4", "int8dyn", "int8dyn_lds"])
def test_split_k_fenced_equals_fence_free(fmt):
    """The default sc1 hand-off (no agent fences) and the fenced memory-model form give
    bit-identical outputs at the maximum split of 8 slices over many tiles."""
    from torchao.kernel import tuning

    M, N, K, g = 32, 4096, 4096, 32
    outs = []
    for fenced in (0, 1, 0):
        if fmt == "int4":
            x, q, s, z, packed, sz = _int4_operands(M, N, K, g, seed=21)
            with tuning(gemm=(16, 1, 8), splitk_fenced=fenced):
                y = torch.ops.torchao.int4_weight_only_linear(x.to(DEV), packed, sz, g, None)
        else:
            w = oracle.make_linear_weight(N, K, seed=22)
            wq, ws = oracle.int8_dyn_weight(w)
            xq, xs = oracle.int8_act_quant(oracle.make_activation(M, K, seed=23))
            knobs = dict(gemm=(64 if fmt == "int8dyn_lds" else 16, 1, 8), splitk_fenced=fenced,
                         gemm_algo=2 if fmt == "int8dyn_lds" else 1)
            with tuning(**knobs):
                y = torch.ops.torchao.int8_scaled_mm(xq.to(DEV), xs.to(DEV), wq.to(DEV),
                                                     ws.to(DEV), None)
        outs.append(y.cpu())
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[0], outs[2])
    if fmt == "int4":
        assert oracle.rel_l2(outs[0], oracle.int4_linear_fp32(x, q, s, z, g)) < TOL_FP32
    else:
        assert torch.equal(outs[0], oracle.int8_scaled_mm(xq, xs, wq, ws, None, epilogue="cpu"))


def test_tuning_is_scoped_and_thread_local():
    """tao_tune_* overrides apply to the calling thread only and tuning() restores defaults."""
    import threading

    from torchao.kernel import tuning

    with pytest.raises(ValueError):
        with tuning(no_such_knob=1):
            pass
    with pytest.raises(RuntimeError, match="splitk_fenced"):
        _lib.call("tao_tune_splitk_fenced", 2)
    _lib.call("tao_tune_reset")
    # an out-of-range override set on another thread must not reach this thread: the crossover
    # forced to 8 there would send M = 6 to the GEMV here; the MFMA path's result differs in bits
    N, K, g = 1024, 2048, 64
    x, q, s, z, packed, sz = _int4_operands(6, N, K, g, seed=31)
    xd = x.to(DEV)
    base = torch.ops.torchao.int4_weight_only_linear(xd, packed, sz, g, None)
    with tuning(linear_crossover=8):
        gemv = torch.ops.torchao.int4_weight_only_linear(xd, packed, sz, g, None)
    t = threading.Thread(target=lambda: _lib.call("tao_tune_linear_crossover", 8))
    t.start()
    t.join()
    after = torch.ops.torchao.int4_weight_only_linear(xd, packed, sz, g, None)
    assert torch.equal(after, base)
    for y in (base, gemv):
        assert oracle.rel_l2(y.cpu(), oracle.int4_linear_fp32(x, q, s, z, g)) < TOL_FP32


@pytest.fixture
def gemm_nw():
    yield lambda nw: _lib.call("tao_tune_gemm_nw", nw)
    _lib.call("tao_tune_gemm_nw", 0)
    _lib.call("tao_tune_gemm", 0, 0, 0)


# 32 columns per wave (tao_tune_gemm_nw 2): every instantiated (bm, kg) with and without split-K,
# ragged N (not a multiple of the 128-column tile) and K tails; the per-element accumulation
# order does not depend on nw, so the outputs equal the 16-column kernel's bit for bit
@pytest.mark.parametrize("bm,kg,splits", [(16, 1, 1), (16, 2, 3), (32, 1, 2), (32, 2, 1),
                                          (64, 1, 4), (64, 2, 1)])
def test_two_column_blocks_per_wave_equal_one(gemm_nw, bm, kg, splits):
    M, N, K, g = 70, 328, 1056, 32
    w = oracle.make_linear_weight(N, K, seed=bm * kg + splits)
    s, z = oracle.int4_qparams(w, g)
    q = oracle.int4_quantize(w, s, z, g)
    x = oracle.make_activation(M, K, seed=splits + 1)
    bias = oracle.make_activation(1, N, seed=6).reshape(N)
    packed = torch.ops.torchao.int4_pack(q.to(DEV))
    sz = torch.stack([s, z], dim=-1).contiguous().to(DEV)
    xd, bd = x.to(DEV), bias.to(DEV)
    s8 = oracle.int8_weight_qparams(w)
    q8 = oracle.int8_weight_quantize(w, s8)
    wq, ws = oracle.int8_dyn_weight(w)
    xq, xs = oracle.int8_act_quant(x)
    _lib.call("tao_tune_gemm", bm, kg, splits)
    _lib.call("tao_tune_gemm_algo", 1)  # int8-dyn on the template kernel
    try:
        outs = {}
        for nw in (1, 2):
            gemm_nw(nw)
            outs[nw] = (
                torch.ops.torchao.int4_weight_only_linear(xd, packed, sz, g, bd).cpu(),
                torch.ops.torchao.int8_weight_only_linear(xd, q8.to(DEV), s8.to(DEV), bd).cpu(),
                torch.ops.torchao.int8_scaled_mm(xq.to(DEV), xs.to(DEV), wq.to(DEV), ws.to(DEV),
                                                 bd).cpu(),
            )
    finally:
        _lib.call("tao_tune_gemm_algo", 0)
    for a, b in zip(outs[1], outs[2]):
        assert torch.equal(a, b)
    assert oracle.rel_l2(outs[2][0], oracle.int4_linear_fp32(x, q, s, z, g, bias)) < TOL_FP32
    assert oracle.rel_l2(outs[2][1], oracle.int8wo_linear(x, q8, s8, bias)) < TOL_REF
    assert torch.equal(outs[2][2], oracle.int8_scaled_mm(xq, xs, wq, ws, bias, epilogue="cpu"))


# entries of the measured shape table (gemm_table.inc) against the heuristic shape and the
# oracle: int4 M=64 6144x4096 (64, 1, 4), int8-wo M=128 28672x4096 (nw 2), int8-dyn M=64
# 6144x4096 (the template kernel in place of the heuristic's), int4 M=100 -> the M=128 bucket,
# int4 M=128 28672x4096 (nw 32: the 32x32x16-MFMA kernel)
@pytest.mark.parametrize("path,M,N,K", [("int4", 64, 6144, 4096), ("int8wo", 128, 28672, 4096),
                                        ("int8dyn", 64, 6144, 4096), ("int4", 100, 6144, 4096),
                                        ("int4", 128, 28672, 4096)])
def test_tuned_shape_table(path, M, N, K):
    g = 32
    w = oracle.make_linear_weight(N, K, seed=N + M)
    x = oracle.make_activation(M, K, seed=M)
    xd = x.to(DEV)
    if path == "int4":
        s, z = oracle.int4_qparams(w, g)
        q = oracle.int4_quantize(w, s, z, g)
        packed = torch.ops.torchao.int4_pack(q.to(DEV))
        sz = torch.stack([s, z], dim=-1).contiguous().to(DEV)
        run = lambda: torch.ops.torchao.int4_weight_only_linear(xd, packed, sz, g, None).cpu()  # noqa: E731
        ref = oracle.int4_linear_fp32(x, q, s, z, g)
    elif path == "int8wo":
        s8 = oracle.int8_weight_qparams(w)
        q8 = oracle.int8_weight_quantize(w, s8)
        run = lambda: torch.ops.torchao.int8_weight_only_linear(xd, q8.to(DEV), s8.to(DEV), None).cpu()  # noqa: E731
        ref = (x.double() @ q8.double().t()) * s8.double()
    else:
        wq, ws = oracle.int8_dyn_weight(w)
        xq, xs = oracle.int8_act_quant(x)
        run = lambda: torch.ops.torchao.int8_scaled_mm(xq.to(DEV), xs.to(DEV), wq.to(DEV), ws.to(DEV), None).cpu()  # noqa: E731
        ref = oracle.int8_scaled_mm(xq, xs, wq, ws, None, epilogue="cpu")
    y_table = run()
    _lib.call("tao_tune_gemm_table", 1)
    try:
        y_heur = run()
    finally:
        _lib.call("tao_tune_gemm_table", 0)
    if path == "int8dyn":
        assert torch.equal(y_table, ref) and torch.equal(y_heur, ref)
    else:
        assert oracle.rel_l2(y_table, ref) < TOL_FP32
        assert oracle.rel_l2(y_table, y_heur) < TOL_FP32


# the int4 GEMM on 32x32x16 MFMAs (tao_tune_int4_mfma32 1): M tiles 32 / 64, split-K, ragged
# N / M / K, every group size, bias; against the oracle's fp32 accumulation of the same weights
@pytest.mark.parametrize("M,N,K,g,bm,splits", [
    (5, 328, 1056, 32, 0, 0), (48, 4096, 1024, 64, 0, 0), (70, 328, 1056, 32, 64, 3),
    (129, 200, 352, 32, 32, 1), (300, 1024, 2048, 128, 64, 2), (128, 4096, 4096, 32, 0, 0),
    (40, 72, 32, 32, 32, 1), (64, 640, 4096, 256, 32, 4)])
def test_int4_mfma32_kernel(M, N, K, g, bm, splits):
    w = oracle.make_linear_weight(N, K, seed=M + K)
    s, z = oracle.int4_qparams(w, g)
    q = oracle.int4_quantize(w, s, z, g)
    x = oracle.make_activation(M, K, seed=M + 1)
    bias = oracle.make_activation(1, N, seed=9).reshape(N)
    packed = torch.ops.torchao.int4_pack(q.to(DEV))
    sz = torch.stack([s, z], dim=-1).contiguous().to(DEV)
    xd, bd = x.to(DEV), bias.to(DEV)
    _lib.call("tao_tune_linear_crossover", 1)
    _lib.call("tao_tune_int4_mfma32", 1)
    _lib.call("tao_tune_gemm", bm, 0, splits)
    try:
        y = torch.ops.torchao.int4_weight_only_linear(xd, packed, sz, g, bd)
        y2 = torch.ops.torchao.int4_weight_only_linear(xd, packed, sz, g, bd)
    finally:
        _lib.call("tao_tune_reset")
    assert torch.equal(y, y2)
    assert oracle.rel_l2(y.cpu(), oracle.int4_linear_fp32(x, q, s, z, g, bias)) < TOL_FP32
    assert oracle.rel_l2(y.cpu(), oracle.int4_linear(x, q, s, z, g, bias)) < TOL_REF
