"""GPU parity of the single-fetch prefill GEMM (csrc/gemm_sf.hip) against the CPU oracle.

128-row tiles (every weight tile fetched by one workgroup), 8 waves, both operands by LDS-DMA into
XOR-swizzled images, K split over workgroups with a fixed reducer (slices 0..S-2 publish sc1
partial tiles and add a ticket; slice S-1 polls it and sums in slice order). Checked here through
the C-ABI (torch.ops.torchao.*): int8 dynamic BIT-EXACT against the reference CPU epilogue
(kernel/intmm.py:133-137, plain_layout.py:301-315) at every tile / wave layout / split / ring
depth / k step; int4 within the reference dequant -> F.linear bar (north star 1e-2) and 4e-3 of
the fp32 accumulation of the same weights at every group size; partial M and N tiles, M > 128
(several M tiles), asymmetric publisher slices, bias, run-to-run bit identity, the fenced
hand-off, agreement with gemm_mfma.hip, graph capture and replay, and no reducer timeouts.
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
def sf():
    def set_(mode, bn=0, wm=0, splits=0, stages=0, a_steps=0, ks=0):
        _lib.call("tao_tune_gemm_sf", mode, bn, wm, splits, stages, a_steps, ks)
    yield set_
    _lib.call("tao_tune_reset")
    st = torch.zeros(1, dtype=torch.int32)
    _lib.call("tao_gemm_sf_status", st.data_ptr())
    assert int(st.item()) == 0, "gemm_sf reducer poll timed out"


def _int4(N, K, g, seed):
    w = oracle.make_linear_weight(N, K, seed=seed)
    s, z = oracle.int4_qparams(w, g)
    q = oracle.int4_quantize(w, s, z, g)
    packed = torch.ops.torchao.int4_pack(q.to(DEV))
    sz = torch.stack([s, z], dim=-1).contiguous().to(DEV)
    return q, s, z, packed, sz


def _int8(M, N, K, seed):
    w = oracle.make_linear_weight(N, K, seed=seed)
    wq, ws = oracle.int8_dyn_weight(w)
    x = oracle.make_activation(M, K, seed=seed + 1)
    xq, xs = oracle.int8_act_quant(x)
    return xq, xs, wq, ws


# (bn, wm, splits, stages, a_steps, ks): every instantiated layout, split 1 / 2 / 4 / 8, ring
# depths 2-4, both int8 k steps
I8_CFGS = [(32, 8, 2, 3, 0, 256), (32, 4, 2, 3, 0, 256), (32, 8, 4, 4, 0, 256),
           (64, 4, 4, 3, 0, 128), (64, 2, 4, 2, 0, 256), (64, 8, 1, 3, 0, 128),
           (128, 2, 8, 2, 0, 128), (128, 4, 2, 4, 0, 128), (64, 4, 2, 3, 0, 256)]
I8_SHAPES = [(128, 4096, 4096), (5, 64, 512), (64, 96, 1024), (100, 4096, 3072),
             (128, 512, 14336), (200, 256, 2048), (1, 128, 256)]


@pytest.mark.parametrize("M,N,K", I8_SHAPES)
@pytest.mark.parametrize("cfg", I8_CFGS)
def test_sf_int8dyn_bit_exact(sf, M, N, K, cfg):
    sf(2, *cfg)
    xq, xs, wq, ws = _int8(M, N, K, seed=M + N + K)
    bias = oracle.make_activation(1, N, seed=3).reshape(N)
    args = (xq.to(DEV), xs.to(DEV), wq.to(DEV), ws.to(DEV))
    y = torch.ops.torchao.int8_scaled_mm(*args, bias.to(DEV)).cpu()
    assert torch.equal(y, oracle.int8_scaled_mm(xq, xs, wq, ws, bias, epilogue="cpu"))
    y = torch.ops.torchao.int8_scaled_mm(*args, None).cpu()
    assert torch.equal(y, oracle.int8_scaled_mm(xq, xs, wq, ws, None, epilogue="cpu"))


def test_sf_int8dyn_extreme_values(sf):
    """Saturated int8 operands (+-127, K = 8192): int32 partials of 127^2 K summed across 4 slices
    stay exact."""
    sf(2, 64, 4, 4, 3, 0, 256)
    M, N, K = 128, 256, 8192
    g = torch.Generator().manual_seed(0)
    wq = (torch.randint(0, 2, (N, K), generator=g, dtype=torch.int8) * 254 - 127).to(torch.int8)
    xq = (torch.randint(0, 2, (M, K), generator=g, dtype=torch.int8) * 254 - 127).to(torch.int8)
    ws = torch.full((N,), 1e-4).to(torch.bfloat16)
    xs = torch.full((M,), 1e-3).to(torch.bfloat16)
    y = torch.ops.torchao.int8_scaled_mm(xq.to(DEV), xs.to(DEV), wq.to(DEV), ws.to(DEV), None).cpu()
    assert torch.equal(y, oracle.int8_scaled_mm(xq, xs, wq, ws, None, epilogue="cpu"))


# (bn, wm, splits, stages, a_steps)
# wm 1: the 32x32x16 kernel (gemm_sf32.hip), 2 or 4 waves of 128 x 32
I4_CFGS = [(64, 2, 4, 3, 0), (64, 4, 4, 3, 0), (64, 8, 2, 2, 0), (128, 2, 8, 2, 0),
           (128, 4, 8, 3, 0), (128, 2, 1, 3, 0), (64, 2, 4, 4, 0), (128, 1, 8, 2, 0),
           (128, 1, 4, 3, 0), (128, 1, 1, 3, 0), (64, 1, 4, 2, 0), (64, 1, 2, 3, 0),
           (256, 1, 1, 3, 0), (256, 1, 2, 2, 0)]  # wm 1, bn 256: 8 waves, 2 per SIMD
I4_SHAPES = [(128, 4096, 4096), (17, 128, 1024), (100, 640, 4096), (128, 512, 14336),
             (200, 192, 2048), (64, 96, 768)]


@pytest.mark.parametrize("M,N,K", I4_SHAPES)
@pytest.mark.parametrize("cfg", I4_CFGS)
def test_sf_int4(sf, M, N, K, cfg):
    sf(2, *cfg)
    g = 32
    q, s, z, packed, sz = _int4(N, K, g, seed=M + N)
    x = oracle.make_activation(M, K, seed=M)
    bias = oracle.make_activation(1, N, seed=7).reshape(N)
    y = torch.ops.torchao.int4_weight_only_linear(x.to(DEV), packed, sz, g, bias.to(DEV)).cpu()
    assert y.shape == (M, N)
    assert oracle.rel_l2(y, oracle.int4_linear(x, q, s, z, g, bias)) < TOL_REF
    assert oracle.rel_l2(y, oracle.int4_linear_fp32(x, q, s, z, g, bias)) < TOL_FP32


@pytest.mark.parametrize("g", [64, 128, 256])
@pytest.mark.parametrize("cfg", [(64, 2, 4, 3, 0), (128, 4, 8, 2, 0), (128, 1, 4, 2, 0),
                                 (64, 1, 2, 3, 0)])
def test_sf_int4_group_sizes(sf, g, cfg):
    """g = 64 / 128 / 256: the (scale, zero) image holds, per 32-k lane group, the word
    ((128 st) >> lg) + ((32 q) >> lg)."""
    sf(2, *cfg)
    M, N, K = 96, 320, 3072
    q, s, z, packed, sz = _int4(N, K, g, seed=g)
    x = oracle.make_activation(M, K, seed=g)
    y = torch.ops.torchao.int4_weight_only_linear(x.to(DEV), packed, sz, g, None).cpu()
    assert oracle.rel_l2(y, oracle.int4_linear_fp32(x, q, s, z, g)) < TOL_FP32
    assert oracle.rel_l2(y, oracle.int4_linear(x, q, s, z, g)) < TOL_REF


@pytest.mark.parametrize("a_steps", [1, 3, 6])
def test_sf_asymmetric_slices(sf, a_steps):
    """Publishers taking fewer (or more) K steps than the reducer: same sums (int8 exact, int4
    within the bars)."""
    M, N, K = 128, 1024, 4096
    sf(2, 32, 8, 2, 3, a_steps, 256)
    xq, xs, wq, ws = _int8(M, N, K, seed=11)
    y = torch.ops.torchao.int8_scaled_mm(xq.to(DEV), xs.to(DEV), wq.to(DEV), ws.to(DEV), None).cpu()
    assert torch.equal(y, oracle.int8_scaled_mm(xq, xs, wq, ws, None, epilogue="cpu"))
    q, s, z, packed, sz = _int4(N, K, 32, seed=12)
    x = oracle.make_activation(M, K, seed=13)
    for wm in (2, 1):
        sf(2, 64, wm, 4, 3, a_steps)
        y = torch.ops.torchao.int4_weight_only_linear(x.to(DEV), packed, sz, 32, None).cpu()
        assert oracle.rel_l2(y, oracle.int4_linear_fp32(x, q, s, z, 32)) < TOL_FP32


@pytest.mark.parametrize("cfg8,cfg4", [((32, 8, 2, 3, 0, 256), (64, 2, 4, 3, 0)),
                                       ((64, 4, 4, 2, 0, 128), (64, 4, 2, 2, 0)),
                                       ((32, 4, 8, 4, 0, 256), (128, 2, 8, 2, 0)),
                                       ((64, 8, 2, 3, 5, 256), (64, 8, 8, 4, 0))])
@pytest.mark.parametrize("M,N,K", [(128, 4096, 4096), (100, 640, 3072), (200, 192, 2048)])
def test_sf_spread_seam_matches_fixed_reducer(sf, cfg8, cfg4, M, N, K):
    """tao_tune_gemm_sf_seam: the spread seam (each of a tile's S workgroups sums 1/S of it) and
    the fixed reducer add the same partials in the same slice order: int8 bit-exact to the
    oracle, int4 bit-identical between the seams (g = 32 and 128) and within the bars; M tiles
    past 128 and ragged N tiles exercise the 1-D grid order."""
    outs = {}
    for seam in (0, 1):
        sf(2, *cfg8)
        _lib.call("tao_tune_gemm_sf_seam", seam)
        xq, xs, wq, ws = _int8(M, N, K, seed=M + K)
        y = torch.ops.torchao.int8_scaled_mm(xq.to(DEV), xs.to(DEV), wq.to(DEV), ws.to(DEV), None).cpu()
        assert torch.equal(y, oracle.int8_scaled_mm(xq, xs, wq, ws, None, epilogue="cpu"))
        sf(2, *cfg4)
        _lib.call("tao_tune_gemm_sf_seam", seam)
        for g in (32, 128):
            q, s, z, packed, sz = _int4(N, K, g, seed=N + g)
            x = oracle.make_activation(M, K, seed=g)
            y = torch.ops.torchao.int4_weight_only_linear(x.to(DEV), packed, sz, g, None).cpu()
            outs.setdefault(g, []).append(y)
            assert oracle.rel_l2(y, oracle.int4_linear_fp32(x, q, s, z, g)) < TOL_FP32
            assert oracle.rel_l2(y, oracle.int4_linear(x, q, s, z, g)) < TOL_REF
    for g, (a, b) in outs.items():
        assert torch.equal(a, b), g


def test_sf_deterministic_fenced_and_matches_old_kernel(sf):
    """Run-to-run bit identity (slices summed in slice order whatever the arrival order), the
    fenced hand-off gives the same bits, and agreement with gemm_mfma.hip (bit-identical for int8
    dyn; fp32 summation orders apart for int4)."""
    M, N, K, g = 128, 4096, 4096, 32
    q, s, z, packed, sz = _int4(N, K, g, seed=1)
    x = oracle.make_activation(M, K, seed=2).to(DEV)
    sf(2, 64, 2, 4, 3)
    a = torch.ops.torchao.int4_weight_only_linear(x, packed, sz, g, None)
    for _ in range(5):
        assert torch.equal(torch.ops.torchao.int4_weight_only_linear(x, packed, sz, g, None), a)
    _lib.call("tao_tune_splitk_fenced", 1)
    assert torch.equal(torch.ops.torchao.int4_weight_only_linear(x, packed, sz, g, None), a)
    _lib.call("tao_tune_splitk_fenced", 0)
    sf(1)
    old = torch.ops.torchao.int4_weight_only_linear(x, packed, sz, g, None)
    assert oracle.rel_l2(a.cpu(), old.cpu()) < 2e-3
    xq, xs, wq, ws = _int8(M, N, K, seed=3)
    args = (xq.to(DEV), xs.to(DEV), wq.to(DEV), ws.to(DEV), None)
    old8 = torch.ops.torchao.int8_scaled_mm(*args)
    sf(2, 32, 8, 2, 3, 0, 256)
    assert torch.equal(torch.ops.torchao.int8_scaled_mm(*args), old8)
    _lib.call("tao_tune_splitk_fenced", 1)
    assert torch.equal(torch.ops.torchao.int8_scaled_mm(*args), old8)


def test_sf_graph_capture(sf):
    """Captured split launches replay correctly (the reducer resets its ticket every launch) and
    recompute on new input."""
    sf(2, 64, 2, 4, 3)
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
    x.copy_(oracle.make_activation(M, K, seed=6).to(DEV))
    graph.replay()
    torch.cuda.synchronize()
    assert torch.equal(out, torch.ops.torchao.int4_weight_only_linear(x, packed, sz, g, None))


def test_sf_unsupported_shapes_fall_back(sf):
    """K not a multiple of the k step (int4 128, int8 256) or an invalid tile choice: the forced
    mode routes to the other kernels, or reports the error."""
    sf(2)
    M, N, K = 64, 256, 1056
    q, s, z, packed, sz = _int4(N, K, 32, seed=N)
    x = oracle.make_activation(M, K, seed=K)
    y = torch.ops.torchao.int4_weight_only_linear(x.to(DEV), packed, sz, 32, None).cpu()
    assert oracle.rel_l2(y, oracle.int4_linear_fp32(x, q, s, z, 32)) < TOL_FP32
    xq, xs, wq, ws = _int8(64, 256, 1152, seed=9)
    y = torch.ops.torchao.int8_scaled_mm(xq.to(DEV), xs.to(DEV), wq.to(DEV), ws.to(DEV), None).cpu()
    assert torch.equal(y, oracle.int8_scaled_mm(xq, xs, wq, ws, None, epilogue="cpu"))
    sf(2, 32, 2)  # bn 32 with 2 waves along M: no kernel (wave tile narrower than 16 columns)
    q, s, z, packed, sz = _int4(256, 1024, 32, seed=1)
    with pytest.raises(RuntimeError, match="gemm_sf"):
        torch.ops.torchao.int4_weight_only_linear(
            oracle.make_activation(64, 1024, seed=1).to(DEV), packed, sz, 32, None)


SW_CFGS = [(0, None), (2, (64, 2, 4, 2, 0)), (2, (64, 2, 2, 3, 0)), (2, (128, 2, 8, 2, 0)),
           (2, (128, 1, 1, 3, 0)), (2, (64, 1, 2, 3, 0)), (2, (128, 1, 4, 2, 0)),
           (2, (256, 1, 1, 3, 0))]


@pytest.mark.parametrize("M,N,K", [(128, 28672, 4096), (100, 1024, 2048), (200, 512, 1024),
                                   (7, 256, 512), (128, 1040, 640)])
@pytest.mark.parametrize("mode,cfg", SW_CFGS)
@pytest.mark.parametrize("seam", [0, 1])
def test_sf_swiglu_epilogue_matches_linear_then_silu_mul(sf, M, N, K, mode, cfg, seam):
    """tao_int4wo_linear_swiglu_bf16 (the w1||w3 GEMM with the SiLU-mul in its epilogue, both
    single-fetch kernels, both seams, partial M and N tiles) is bit-identical to the
    routed linear followed by tao_silu_mul_bf16 on the same launch shape; where no fused kernel
    serves the shape (auto routing off the measured shapes) the wrapper returns None."""
    from torchao._models.llama import kernels

    sf(mode, *(cfg or ()))
    _lib.call("tao_tune_gemm_sf_seam", seam)
    q, s, z, packed, sz = _int4(N, K, 32, seed=N + K)
    x = oracle.make_activation(M, K, seed=M).to(DEV)
    y = kernels.int4_linear_swiglu(x, packed, sz, 32)
    if M > 128 or (mode == 0 and (M, N, K) != (128, 28672, 4096)):
        assert y is None  # the single-fetch GEMM serves one 128-row tile per launch
        return
    assert y is not None and y.shape == (M, N // 2)
    ref = kernels.silu_mul(torch.ops.torchao.int4_weight_only_linear(x, packed, sz, 32, None))
    assert torch.equal(y, ref)


@pytest.mark.parametrize("B,S,H,Hkv,K,p0,T", [(1, 128, 32, 8, 4096, 0, 200), (1, 100, 4, 2, 512, 7, 160),
                                              (2, 50, 4, 1, 1024, 0, 64)])
@pytest.mark.parametrize("mode,cfg", [(0, None), (2, (64, 2, 4, 2, 0)), (2, (128, 2, 2, 3, 0)),
                                      (2, (64, 4, 1, 3, 0))])
@pytest.mark.parametrize("seam", [0, 1])
def test_sf_rope_kv_epilogue_matches_linear_then_rope_kv(sf, B, S, H, Hkv, K, p0, T, mode, cfg,
                                                        seam):
    """tao_int4wo_linear_rope_kv_bf16 (wqkv GEMM with RoPE + the KV-cache write in its epilogue)
    writes the same q and cache rows, bit for bit, as the routed linear followed by
    tao_rope_kv_bf16; cache rows outside the prompt's positions stay untouched; shapes no fused
    kernel serves return None."""
    import math

    from torchao._models.llama import kernels
    from torchao._models.llama.model import ModelArgs, _rope_freqs

    sf(mode, *(cfg or ()))
    _lib.call("tao_tune_gemm_sf_seam", seam)
    D = 128
    N = (H + 2 * Hkv) * D
    q, s_, z, packed, sz = _int4(N, K, 32, seed=N + K + S)
    x = oracle.make_activation(B * S, K, seed=S).reshape(B, S, K).to(DEV)
    freqs = _rope_freqs(ModelArgs(dim=H * D, n_head=H, n_local_heads=Hkv, block_size=T), T).to(DEV)
    pos = torch.arange(p0, p0 + S, device=DEV)
    kc = [torch.full((B, Hkv, T, D), 7, dtype=torch.bfloat16, device=DEV) for _ in range(2)]
    vc = [torch.full((B, Hkv, T, D), 7, dtype=torch.bfloat16, device=DEV) for _ in range(2)]
    got = kernels.int4_linear_rope_kv(x, packed, sz, 32, freqs, pos, kc[0], vc[0], H)
    if B * S > 128 or (mode == 0 and (N, K) != (6144, 4096)) or (mode == 0 and B * S <= 64):
        assert got is None
        return
    assert got is not None
    qkv = torch.ops.torchao.int4_weight_only_linear(x.reshape(B * S, K), packed, sz, 32, None)
    ref = kernels.rope_kv(qkv.reshape(B, S, N), freqs, pos, kc[1], vc[1], H)
    assert torch.equal(got, ref)
    assert torch.equal(kc[0], kc[1]) and torch.equal(vc[0], vc[1])
    assert bool((kc[0][:, :, p0 + S:] == 7).all()) and bool((kc[0][:, :, :p0] == 7).all())
    assert not math.isnan(float(got.float().sum()))


def test_sf_rope_kv_epilogue_position_past_cache(sf):
    """A prompt position outside [0, T) writes no cache row and sets tao_decode_status bit 1,
    as tao_rope_kv_bf16 does."""
    from torchao._models.llama import kernels
    from torchao._models.llama.model import ModelArgs, _rope_freqs

    sf(2, 64, 2, 2, 3, 0)
    H, Hkv, D, K, S, T = 4, 2, 128, 512, 8, 16
    N = (H + 2 * Hkv) * D
    _, _, _, packed, sz = _int4(N, K, 32, seed=5)
    x = oracle.make_activation(S, K, seed=2).reshape(1, S, K).to(DEV)
    freqs = _rope_freqs(ModelArgs(dim=H * D, n_head=H, n_local_heads=Hkv, block_size=64), 64).to(DEV)
    pos = torch.arange(12, 12 + S, device=DEV)  # rows 16.. are past the cache
    kc = torch.full((1, Hkv, T, D), 7, dtype=torch.bfloat16, device=DEV)
    vc = kc.clone()
    st = torch.zeros(1, dtype=torch.int32)
    _lib.call("tao_decode_status", st.data_ptr())  # clear
    assert kernels.int4_linear_rope_kv(x, packed, sz, 32, freqs, pos, kc, vc, H) is not None
    torch.cuda.synchronize()
    _lib.call("tao_decode_status", st.data_ptr())
    assert int(st.item()) & 1
    assert bool((kc[:, :, :12] == 7).all()) and bool((kc[:, :, 12:16] != 7).any())


def test_sf_swiglu_prefill_model_matches_unfused():
    """A small Llama prefill (dim 512, head_dim 128, w1||w3 3072 x 512) with the SwiGLU folded
    into the w1||w3 GEMM and RoPE + the KV write folded into the wqkv GEMM (every linear on the
    single-fetch kernel) gives bit-identical hidden states and caches to the linear + silu_mul /
    rope_kv path on the same kernels."""
    import math

    from torchao._models.llama import model as mdl
    from torchao._models.llama.generate import apply_quantization
    from torchao._models.llama.model import ModelArgs, Transformer
    from torchao.kernel import tuning

    dev = torch.device(DEV)
    torch.manual_seed(7)
    m = Transformer(ModelArgs(dim=512, n_layer=2, n_head=4, n_local_heads=2, vocab_size=1000,
                              block_size=256)).to(dev).to(torch.bfloat16)
    with torch.no_grad():
        for mod in m.modules():
            if isinstance(mod, torch.nn.Linear):
                b = 1 / math.sqrt(mod.in_features)
                mod.weight.uniform_(-b, b)
    m.fuse_w13()
    apply_quantization(m, "int4wo-32")
    m.setup_caches(1, 160)
    assert m.enable_fused_kernels()
    idx = torch.randint(0, 1000, (1, 128), device=dev,
                        generator=torch.Generator(device=dev).manual_seed(1))
    pos = torch.arange(128, device=dev)
    outs = []
    with tuning(gemm_sf=(2, 0, 0, 0, 0, 0, 0)):
        ff = m.layers[0].feed_forward
        assert ff.swiglu_prefill is not None and mdl._int4_parts(ff.w13) is not None
        from torchao._models.llama import kernels

        assert kernels.int4_linear_swiglu(torch.zeros(128, 512, device=dev, dtype=torch.bfloat16),
                                          *mdl._int4_parts(ff.w13)) is not None
        assert kernels.int4_linear_rope_kv(
            torch.zeros(1, 128, 512, device=dev, dtype=torch.bfloat16),
            *mdl._int4_parts(m.layers[0].attention.wqkv), m.freqs, pos,
            m.layers[0].attention.kv_cache.k_cache.clone(),
            m.layers[0].attention.kv_cache.v_cache.clone(), 4) is not None
        for fused in (True, False):
            mdl.PREFILL_SWIGLU = mdl.PREFILL_ROPE = fused
            try:
                outs.append(m._layers_prefill(idx, pos).clone())
                outs.append(m.layers[1].attention.kv_cache.k_cache.clone())
            finally:
                mdl.PREFILL_SWIGLU = mdl.PREFILL_ROPE = True
    assert torch.equal(outs[0], outs[2]) and torch.equal(outs[1], outs[3])


@pytest.mark.parametrize("cfg8,cfg4", [((256, 2, 2, 2, 0, 128), (256, 2, 2, 2, 0)),
                                       ((256, 4, 1, 3, 0, 128), (256, 4, 4, 3, 0)),
                                       ((256, 2, 4, 3, 0, 128), (256, 2, 1, 3, 0))])
@pytest.mark.parametrize("M,N,K", [(128, 4096, 4096), (100, 640, 3072), (200, 288, 2048)])
def test_sf_bn256(sf, cfg8, cfg4, M, N, K):
    """256-column tiles (x read once per 256 weight columns): int8 dyn bit-exact, int4 within the
    bars at g = 32 and 128, ragged N tiles and several M tiles, both seams."""
    for seam in (0, 1):
        sf(2, *cfg8)
        _lib.call("tao_tune_gemm_sf_seam", seam)
        xq, xs, wq, ws = _int8(M, N, K, seed=M + K)
        y = torch.ops.torchao.int8_scaled_mm(xq.to(DEV), xs.to(DEV), wq.to(DEV), ws.to(DEV), None).cpu()
        assert torch.equal(y, oracle.int8_scaled_mm(xq, xs, wq, ws, None, epilogue="cpu"))
        sf(2, *cfg4)
        _lib.call("tao_tune_gemm_sf_seam", seam)
        for g in (32, 128):
            q, s, z, packed, sz = _int4(N, K, g, seed=N + g)
            x = oracle.make_activation(M, K, seed=g)
            y = torch.ops.torchao.int4_weight_only_linear(x.to(DEV), packed, sz, g, None).cpu()
            assert oracle.rel_l2(y, oracle.int4_linear_fp32(x, q, s, z, g)) < TOL_FP32
            assert oracle.rel_l2(y, oracle.int4_linear(x, q, s, z, g)) < TOL_REF


@pytest.mark.parametrize("cfg", [(128, 1, 1, 3, 0, 2), (128, 1, 4, 2, 0, 2), (128, 1, 2, 3, 0, 2),
                                 (128, 1, 8, 2, 3, 2)])
@pytest.mark.parametrize("M,N,K", [(128, 4096, 4096), (100, 640, 3072), (200, 384, 2048),
                                   (128, 28672, 4096)])
def test_sf32_k_halves(sf, cfg, M, N, K):
    """The 32x32x16 int4 kernel with two waves per column group splitting each step's k (summed
    through LDS in k-half order): within the bars at g = 32 and 128, run-to-run identical, and its
    SwiGLU epilogue bit-identical to the linear + silu_mul on the same shape."""
    from torchao._models.llama import kernels

    sf(2, *cfg)
    for g in (32, 128):
        q, s, z, packed, sz = _int4(N, K, g, seed=N + g)
        x = oracle.make_activation(M, K, seed=g)
        xd = x.to(DEV)
        y = torch.ops.torchao.int4_weight_only_linear(xd, packed, sz, g, None)
        assert torch.equal(y, torch.ops.torchao.int4_weight_only_linear(xd, packed, sz, g, None))
        if N <= 4096:
            yc = y.cpu()
            assert oracle.rel_l2(yc, oracle.int4_linear_fp32(x, q, s, z, g)) < TOL_FP32
            assert oracle.rel_l2(yc, oracle.int4_linear(x, q, s, z, g)) < TOL_REF
        if M <= 128:
            sw = kernels.int4_linear_swiglu(xd, packed, sz, g)
            assert sw is not None and torch.equal(sw, kernels.silu_mul(y))


@pytest.mark.parametrize("cfg", [(128, 1, 1, 3, 0, 0), (128, 1, 4, 3, 0, 0), (64, 1, 2, 3, 0, 0),
                                 (128, 1, 2, 3, 5, 0), (128, 1, 1, 3, 0, 2), (128, 1, 4, 3, 0, 2),
                                 (128, 1, 2, 3, 5, 2)])
@pytest.mark.parametrize("M,N,K", [(128, 4096, 4096), (100, 640, 3072), (200, 384, 2048),
                                   (128, 28672, 4096), (1, 96, 512)])
def test_sf32_loader_waves_bit_identical(sf, cfg, M, N, K):
    """Dedicated LDS-DMA loader waves (tao_tune_gemm_sf_loaders 2) change who issues the DMA
    pieces and when, not what any compute wave reads or sums: outputs bit-identical to the
    kernel without them, its SwiGLU epilogue too, at g = 32 (16-B (scale, zero) pieces) and 128
    (4-B pieces), split or not, ragged M / N, several M tiles; one or two compute waves per
    column group (k halves, ks 2)."""
    from torchao._models.llama import kernels

    sf(2, *cfg)
    for g in (32, 128):
        q, s, z, packed, sz = _int4(N, K, g, seed=N + g)
        x = oracle.make_activation(M, K, seed=g).to(DEV)
        _lib.call("tao_tune_gemm_sf_loaders", 1)
        ref = torch.ops.torchao.int4_weight_only_linear(x, packed, sz, g, None)
        ref_sw = kernels.int4_linear_swiglu(x, packed, sz, g) if M <= 128 else None
        _lib.call("tao_tune_gemm_sf_loaders", 2)
        got = torch.ops.torchao.int4_weight_only_linear(x, packed, sz, g, None)
        assert torch.equal(got, ref)
        if ref_sw is not None:
            assert torch.equal(kernels.int4_linear_swiglu(x, packed, sz, g), ref_sw)
        if N <= 4096:
            assert oracle.rel_l2(got.cpu(), oracle.int4_linear(x.cpu(), q, s, z, g)) < TOL_REF


@pytest.mark.parametrize("seam", [0, 1])
@pytest.mark.parametrize("cfg", [(64, 2, 4, 2, 0, 0), (64, 4, 1, 3, 0, 0), (64, 8, 2, 4, 0, 0),
                                 (64, 2, 8, 3, 0, 0)])
@pytest.mark.parametrize("M,N,K", [(128, 4096, 4096), (100, 640, 3072), (200, 384, 2048),
                                   (1, 96, 512)])
def test_sf16_loader_waves_bit_identical(sf, seam, cfg, M, N, K):
    """The 16x16x32 kernel with 4 dedicated LDS-DMA loader waves beside its 8 compute waves
    (tao_tune_gemm_sf_loaders 2, 64-column tiles): int4 (g 32 / 128) and int8 dynamic outputs
    bit-identical to the kernel whose compute waves issue the DMA pieces themselves, under both
    split-K seams (fixed reducer, spread)."""
    sf(2, *cfg)
    _lib.call("tao_tune_gemm_sf_seam", seam)
    for g in (32, 128):
        q, s, z, packed, sz = _int4(N, K, g, seed=N + g)
        x = oracle.make_activation(M, K, seed=g).to(DEV)
        _lib.call("tao_tune_gemm_sf_loaders", 1)
        ref = torch.ops.torchao.int4_weight_only_linear(x, packed, sz, g, None)
        _lib.call("tao_tune_gemm_sf_loaders", 2)
        got = torch.ops.torchao.int4_weight_only_linear(x, packed, sz, g, None)
        assert torch.equal(got, ref)
    xq, xs, wq, ws = (t.to(DEV) for t in _int8(M, N, K, seed=M + N))
    sf(2, *cfg[:5], 128)
    _lib.call("tao_tune_gemm_sf_loaders", 1)
    ref = torch.ops.torchao.int8_scaled_mm(xq, xs, wq, ws, None)
    _lib.call("tao_tune_gemm_sf_loaders", 2)
    got = torch.ops.torchao.int8_scaled_mm(xq, xs, wq, ws, None)
    assert torch.equal(got, ref)
    assert torch.equal(got.cpu(), oracle.int8_scaled_mm(xq.cpu(), xs.cpu(), wq.cpu(), ws.cpu(),
                                                       None, epilogue="cpu"))


@pytest.mark.parametrize("cfg", [(64, 2, 4, 2, 0, 0), (64, 4, 2, 3, 0, 0), (128, 2, 8, 2, 0, 0),
                                 (64, 2, 4, 4, 3, 0)])
@pytest.mark.parametrize("M,N,K", [(128, 4096, 4096), (200, 1024, 2048), (100, 4096, 14336)])
def test_sf_xcd_slice_map_bit_identical(sf, cfg, M, N, K):
    """K slice -> XCD placement (tao_tune_gemm_sf_xmap 2) only renumbers the workgroups: int4 and
    int8 dynamic outputs bit-identical to the default numbering, asymmetric slices and several
    M tiles included; N / 64 not a multiple of 8 / S falls back to the default numbering."""
    sf(2, *cfg)
    _lib.call("tao_tune_gemm_sf_seam", 0)
    q, s, z, packed, sz = _int4(N, K, 32, seed=N)
    x = oracle.make_activation(M, K, seed=5).to(DEV)
    _lib.call("tao_tune_gemm_sf_xmap", 1)
    ref = torch.ops.torchao.int4_weight_only_linear(x, packed, sz, 32, None)
    _lib.call("tao_tune_gemm_sf_xmap", 2)
    assert torch.equal(torch.ops.torchao.int4_weight_only_linear(x, packed, sz, 32, None), ref)
    xq, xs, wq, ws = (t.to(DEV) for t in _int8(M, N, K, seed=M + N))
    sf(2, *cfg[:5], 128)
    _lib.call("tao_tune_gemm_sf_xmap", 1)
    ref = torch.ops.torchao.int8_scaled_mm(xq, xs, wq, ws, None)
    _lib.call("tao_tune_gemm_sf_xmap", 2)
    got = torch.ops.torchao.int8_scaled_mm(xq, xs, wq, ws, None)
    assert torch.equal(got, ref)
    assert torch.equal(got.cpu(), oracle.int8_scaled_mm(xq.cpu(), xs.cpu(), wq.cpu(), ws.cpu(),
                                                       None, epilogue="cpu"))


@pytest.mark.parametrize("path,cfg", [("int4", (64, 2, 4, 2, 0, 0)), ("int4", (128, 1, 4, 3, 0, 0)),
                                      ("int8", (64, 4, 4, 3, 0, 128))])
def test_sf_reducer_timeout_recovers(sf, path, cfg):
    """A split-K launch whose reducers time out (tao_debug_sf_late_publisher: slice-0 publishers
    add their ticket only after a reducer gave up) is reported through tao_decode_status (bits & 2),
    and leaves every tile's ticket at 0: the following launches on the same stream's workspace
    are bit-identical to the ones before it, and report nothing."""
    sf(2, *cfg)
    _lib.call("tao_tune_gemm_sf_seam", 0)
    M, N, K = 128, 512, 2048
    if path == "int4":
        q, s, z, packed, sz = _int4(N, K, 32, seed=11)
        x = oracle.make_activation(M, K, seed=12).to(DEV)

        def run():
            return torch.ops.torchao.int4_weight_only_linear(x, packed, sz, 32, None)
    else:
        xq, xs, wq, ws = (t.to(DEV) for t in _int8(M, N, K, seed=13))

        def run():
            return torch.ops.torchao.int8_scaled_mm(xq, xs, wq, ws, None)
    bits = torch.zeros(1, dtype=torch.int32)
    ref = run()
    torch.cuda.synchronize()
    _lib.call("tao_decode_status", bits.data_ptr())
    assert int(bits.item()) == 0
    _lib.call("tao_debug_sf_late_publisher", 1)
    try:
        run()
        torch.cuda.synchronize()
    finally:
        _lib.call("tao_debug_sf_late_publisher", 0)
    _lib.call("tao_decode_status", bits.data_ptr())
    assert int(bits.item()) & 2, "timed-out reducers were not reported"
    for _ in range(3):
        assert torch.equal(run(), ref)
    torch.cuda.synchronize()
    _lib.call("tao_decode_status", bits.data_ptr())
    assert int(bits.item()) == 0


@pytest.mark.parametrize("cfg", [None, (64, 2, 1, 3, 0, 0), (64, 2, 2, 3, 0, 0), (64, 4, 4, 2, 0, 0),
                                 (64, 2, 8, 3, 5, 0), (128, 2, 4, 3, 0, 0)])
@pytest.mark.parametrize("M,N,K", [(128, 4096, 4096), (100, 640, 3072), (128, 4096, 14336),
                                   (77, 512, 2048)])
def test_sf_partials_then_add_rmsnorm_bit_identical(sf, cfg, M, N, K):
    """The prefill's wo / w2 without an in-kernel split-K seam: every K slice writes its fp32
    partial tile (int4_linear_partials) and the residual add + RMSNorm sums them in slice order
    (add_rmsnorm_partials): h and y bit-identical to add_rmsnorm(x, linear(...)) on the same
    launch shape, whatever the split (1-8 slices, uneven slices, several M tiles, ragged M)."""
    from torchao._models.llama import kernels

    if cfg is None:  # the built-in route (served at M = 128 for the two Llama shapes only)
        if M != 128 or N != 4096:
            pytest.skip("no built-in route")
    else:
        sf(2, *cfg)
    q, s, z, packed, sz = _int4(N, K, 32, seed=N + K)
    a = oracle.make_activation(M, K, seed=M).to(DEV)
    x = oracle.make_activation(M, N, seed=M + 1).to(DEV)
    w = (torch.rand(N, generator=torch.Generator().manual_seed(3)) + 0.5).to(torch.bfloat16).to(DEV)
    part = kernels.int4_linear_partials(a, packed, sz, 32)
    assert part is not None and part.shape[1:] == (M, N)
    lin = torch.ops.torchao.int4_weight_only_linear(a, packed, sz, 32, None)
    h0, y0 = kernels.add_rmsnorm(x, lin, w, 1e-5)
    h1, y1 = kernels.add_rmsnorm_partials(x, part, w, 1e-5)
    assert torch.equal(h1, h0) and torch.equal(y1, y0)


def test_sf_partials_not_served_on_the_32x32_route(sf):
    """Shapes routed to the 32x32x16 kernel (one wave along M) have no partials-out form: None,
    and the caller keeps the plain linear."""
    from torchao._models.llama import kernels

    sf(2, 128, 1, 2, 3, 0, 0)
    q, s, z, packed, sz = _int4(512, 1024, 32, seed=9)
    a = oracle.make_activation(128, 1024, seed=1).to(DEV)
    assert kernels.int4_linear_partials(a, packed, sz, 32) is None


def _rand_cases(seed, n):
    """Seeded random (M, N, K, launch shape) cases for the single-fetch GEMMs."""
    import random

    r = random.Random(seed)
    out = []
    for _ in range(n):
        M = r.choice([1, 7, 33, 64, 65, 100, 127, 128])
        N = 64 * r.randint(1, 24) + r.choice([0, 0, 16, 48])
        K = 128 * r.randint(2, 24)
        bn = r.choice([64, 64, 128])
        wm = r.choice([2, 4, 8]) if bn == 64 else r.choice([2, 4])
        S = r.choice([1, 2, 4, 8])
        stages = r.choice([2, 3, 4]) if bn == 64 else r.choice([2, 3])
        out.append((M, N, K, (bn, wm, S, stages, 0, 0)))
    return out


@pytest.mark.parametrize("case", _rand_cases(2025, 24))
def test_sf_random_shapes_all_forms_agree(sf, case):
    """Seeded random shapes and launch shapes through every int4 form of the 16x16 single-fetch
    GEMM that round 5 added beside the plain one: loader waves (4 DMA waves, 64-column tiles),
    the K-slice -> XCD numbering, and the partials-out epilogue summed by add_rmsnorm_partials:
    each bit-identical to the plain launch of the same shape, which is within the oracle bar."""
    from torchao._models.llama import kernels

    M, N, K, cfg = case
    sf(2, *cfg)
    _lib.call("tao_tune_gemm_sf_seam", 0)
    q, s, z, packed, sz = _int4(N, K, 32, seed=N * 7 + K)
    a = oracle.make_activation(M, K, seed=M + K).to(DEV)
    _lib.call("tao_tune_gemm_sf_loaders", 1)
    ref = torch.ops.torchao.int4_weight_only_linear(a, packed, sz, 32, None)
    if cfg[0] == 64:
        _lib.call("tao_tune_gemm_sf_loaders", 2)
        assert torch.equal(torch.ops.torchao.int4_weight_only_linear(a, packed, sz, 32, None), ref)
        _lib.call("tao_tune_gemm_sf_loaders", 1)
    _lib.call("tao_tune_gemm_sf_xmap", 2)
    assert torch.equal(torch.ops.torchao.int4_weight_only_linear(a, packed, sz, 32, None), ref)
    _lib.call("tao_tune_gemm_sf_xmap", 1)
    part = kernels.int4_linear_partials(a, packed, sz, 32)
    if M <= 2:  # the plain linear runs the skinny-M GEMV there: no partials form
        assert part is None
    elif N % 8 == 0:
        assert part is not None
        x = oracle.make_activation(M, N, seed=3).to(DEV)
        w = torch.ones(N, dtype=torch.bfloat16, device=DEV)
        h0, y0 = kernels.add_rmsnorm(x, ref, w, 1e-5)
        h1, y1 = kernels.add_rmsnorm_partials(x, part, w, 1e-5)
        assert torch.equal(h1, h0) and torch.equal(y1, y0)
    if N * K <= 4096 * 4096:
        assert oracle.rel_l2(ref.cpu(), oracle.int4_linear(a.cpu(), q, s, z, 32)) < TOL_REF


@pytest.mark.parametrize("path", [0, 2])
def test_sf_intake_probe_runs_the_launch_shape(sf, path):
    """bench.py's intake ceiling (tao_sf_intake_probe): the probe streams the launch shape the GEMM
    takes at 128 x 4096 x 4096 (the int4 route: 64-column tiles, 4 K slices, 4 stages, 4 loader
    waves; int8 dyn: the single-fetch default) and reports it; it rejects M outside one tile."""
    import ctypes

    M, N, K, g = 128, 4096, 4096, 32
    if path == 0:
        q, s, z, packed, sz = _int4(N, K, g, seed=5)
        x = oracle.make_activation(M, K, seed=6).to(DEV)
        w, zz = packed, sz
    else:
        x, _, w, _ = (t.to(DEV) for t in _int8(M, N, K, seed=7))
        zz = None
    shp = (ctypes.c_int * 7)()
    sink = torch.zeros(1024, dtype=torch.int32, device=DEV)
    h = _lib.lib()

    def run(m):
        return h.tao_sf_intake_probe(path, 0, x.data_ptr(), w.data_ptr(),
                                     zz.data_ptr() if zz is not None else None, m, N, K, g,
                                     ctypes.cast(shp, ctypes.c_void_p), sink.data_ptr(),
                                     torch.cuda.current_stream().cuda_stream)

    assert run(M) == 0
    torch.cuda.synchronize()
    bn, S, ns, a, ld, ks, step_b = list(shp)
    if path == 0:
        assert (bn, S, ns, a, ld, ks) == (64, 4, 4, 8, 4, 128)
        assert step_b == 128 * 256 + 64 * 64 + 64 * 16
    else:
        assert ks in (128, 256) and step_b == 128 * ks + bn * ks and S * a <= K // ks
    assert int(sink.sum().item()) == 0
    assert run(32) != 0  # one 128-row tile only
