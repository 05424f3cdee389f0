"""The decode-fused int8 GEMVs (tao_int8wo_decode_bf16, and tao_int8dq_decode_bf16 for the
dynamic-activation config) against the unfused chain they replace: RMSNorm kernel -> int8
linear -> SiLU-mul / RoPE + KV write. Without the RMSNorm prologue the outputs are the linear's
own bf16(bf16(sum) * scale) values: int8-dyn sums are exact integers (bit-exact), int8 weight-only
sums may differ in fp32 order from the unfused launch shape. With the prologue, the sum of
squares inside rsqrt(mean(x^2) + eps) may round differently, so a normalised activation may
differ by one bf16 ulp (tolerance per check). Also checked against the fp32 chain at the
north-star bar (1e-2)."""

import math

import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from torchao.quantization import (
    Int8DynamicActivationInt8WeightConfig,
    Int8WeightOnlyConfig,
    quantize_,
)

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _int8_linear(N, K, seed=0):
    torch.manual_seed(seed)
    lin = nn.Linear(K, N, bias=False, device=DEV, dtype=torch.bfloat16)
    with torch.no_grad():
        lin.weight.uniform_(-1 / math.sqrt(K), 1 / math.sqrt(K))
    quantize_(lin, Int8WeightOnlyConfig())
    from torchao._models.llama.model import _int8wo_parts

    parts = _int8wo_parts(lin)
    assert parts is not None
    return lin, parts


def _norm_w(K, seed=1):
    g = torch.Generator(device=DEV).manual_seed(seed)
    return (torch.rand(K, device=DEV, generator=g) + 0.5).to(torch.bfloat16)


def _rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm())


@pytest.mark.parametrize("N,K", [(512, 4096), (6144, 4096), (4096, 14336), (1000, 512),
                                 (8192, 8192), (128256, 4096)])
def test_plain_matches_linear(N, K):
    from torchao._models.llama import kernels

    lin, parts = _int8_linear(N, K)
    x = torch.randn(1, 1, K, device=DEV, dtype=torch.bfloat16)
    got = kernels.int8wo_decode(x, *parts)
    ref = lin(x)
    assert got.shape == ref.shape
    assert _rel(got, ref) < 2e-3
    # the fp32 chain: x @ (q * s)^T
    impl = lin.weight.tensor_impl
    w32 = impl.int_data.float() * impl.scale.reshape(-1, 1).float()
    assert _rel(got, F.linear(x.float(), w32)) < 1e-2


@pytest.mark.parametrize("N,K", [(512, 4096), (6144, 4096), (128256, 4096), (2048, 8192)])
def test_rmsnorm_prologue(N, K):
    from torchao._models.llama import kernels

    lin, parts = _int8_linear(N, K)
    x = torch.randn(1, 1, K, device=DEV, dtype=torch.bfloat16) * 3
    w = _norm_w(K)
    got = kernels.int8wo_decode(x, *parts, norm_weight=w, eps=1e-5)
    ref = lin(kernels.rmsnorm(x, w, 1e-5))
    assert _rel(got, ref) < 3e-3
    xf = x.float()
    xn = (xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + 1e-5)).bfloat16() * w
    impl = lin.weight.tensor_impl
    w32 = impl.int_data.float() * impl.scale.reshape(-1, 1).float()
    assert _rel(got, F.linear(xn.float(), w32)) < 1e-2


@pytest.mark.parametrize("norm", [False, True])
@pytest.mark.parametrize("I,K", [(256, 512), (14336, 4096)])
def test_swiglu_epilogue(norm, I, K):
    from torchao._models.llama import kernels

    lin, parts = _int8_linear(2 * I, K, seed=2)  # rows interleaved (gate_i, up_i)
    x = torch.randn(1, 1, K, device=DEV, dtype=torch.bfloat16)
    w = _norm_w(K) if norm else None
    got = kernels.int8wo_decode(x, *parts, norm_weight=w, eps=1e-5, epilogue="swiglu")
    assert got.shape == (1, 1, I)
    xin = kernels.rmsnorm(x, w, 1e-5) if norm else x
    ref = kernels.silu_mul(lin(xin))
    assert _rel(got, ref) < 3e-3


@pytest.mark.parametrize("norm", [False, True])
@pytest.mark.parametrize("H,Hkv,pos", [(32, 8, 17), (4, 4, 0), (8, 2, 63)])
def test_rope_kv_epilogue(norm, H, Hkv, pos):
    from torchao._models.llama import kernels
    from torchao._models.llama.model import ModelArgs, _rope_freqs

    D, T = 128, 64
    K = 1024 if H < 32 else 4096
    N = (H + 2 * Hkv) * D
    lin, parts = _int8_linear(N, K, seed=3)
    cfg = ModelArgs(n_layer=1, n_head=H, n_local_heads=Hkv, dim=H * D, rope_base=500000)
    freqs = _rope_freqs(cfg, T).to(DEV)
    x = torch.randn(1, 1, K, device=DEV, dtype=torch.bfloat16)
    w = _norm_w(K) if norm else None
    p = torch.tensor([pos], device=DEV)
    kc = torch.randn(1, Hkv, T, D, device=DEV, dtype=torch.bfloat16)
    vc = torch.randn_like(kc)
    kc_ref, vc_ref = kc.clone(), vc.clone()
    q = kernels.int8wo_decode(x, *parts, norm_weight=w, eps=1e-5, epilogue="rope_kv",
                              rope=(freqs, p, kc, vc, H))
    xin = kernels.rmsnorm(x, w, 1e-5) if norm else x
    q_ref = kernels.rope_kv(lin(xin), freqs, p, kc_ref, vc_ref, H)
    for a, b in ((q, q_ref), (kc, kc_ref), (vc, vc_ref)):
        assert _rel(a, b) < 3e-3
    rows = [t for t in range(T) if t != pos]
    assert torch.equal(kc[:, :, rows], kc_ref[:, :, rows])  # other rows untouched
    assert torch.equal(vc[:, :, rows], vc_ref[:, :, rows])


def test_graph_capture_errors_and_kv_guard():
    from torchao import _lib
    from torchao._models.llama import kernels
    from torchao._models.llama.model import ModelArgs, _rope_freqs

    lin, parts = _int8_linear(6144, 4096)
    x = torch.randn(1, 1, 4096, device=DEV, dtype=torch.bfloat16)
    w = _norm_w(4096)
    eager = kernels.int8wo_decode(x, *parts, norm_weight=w, eps=1e-5)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        kernels.int8wo_decode(x, *parts, norm_weight=w, eps=1e-5)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            out = kernels.int8wo_decode(x, *parts, norm_weight=w, eps=1e-5)
    torch.cuda.current_stream().wait_stream(s)
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(out, eager)
    with pytest.raises(RuntimeError, match="one token"):
        kernels.int8wo_decode(torch.randn(2, 4096, device=DEV, dtype=torch.bfloat16), *parts)
    with pytest.raises(RuntimeError, match="epilogue"):
        _lib.call("tao_int8wo_decode_bf16", x.data_ptr(), parts[0].data_ptr(),
                  parts[1].data_ptr(), 6144, 4096, None, 0.0, 7, eager.data_ptr(), None, None,
                  None, None, 0, 0, 0, 0, None)
    # a KV position past the cache: no row written, reported by tao_decode_status
    H, Hkv, D, T = 32, 8, 128, 16
    cfg = ModelArgs(n_layer=1, n_head=H, n_local_heads=Hkv, dim=H * D, rope_base=500000)
    freqs = _rope_freqs(cfg, 64).to(DEV)
    kc = torch.zeros(1, Hkv, T, D, device=DEV, dtype=torch.bfloat16)
    vc = torch.zeros_like(kc)
    kernels.check_decode_status()  # clear
    kernels.int8wo_decode(x, *parts, epilogue="rope_kv",
                          rope=(freqs, torch.tensor([T], device=DEV), kc, vc, H))
    torch.cuda.synchronize()
    assert not kc.any() and not vc.any()
    with pytest.raises(RuntimeError):
        kernels.check_decode_status()


@pytest.mark.parametrize("quant", ["int8wo", "int8dq"])
def test_fused_int8_decode_in_the_harness(quant):
    """A tiny Llama on Int8WeightOnlyConfig: the fused one-token step (norms, RoPE + KV and
    SwiGLU inside the int8 GEMVs) tracks the torch-op step, and a HIP-graph replay equals it."""
    from torchao._models.llama.generate import GraphDecoder, apply_quantization, generate, prefill
    from torchao._models.llama.model import ModelArgs, Transformer

    torch.manual_seed(2)
    model = Transformer(ModelArgs(dim=512, n_layer=2, n_head=4, n_local_heads=2, vocab_size=1000,
                                  block_size=256)).to(DEV).to(torch.bfloat16)
    with torch.no_grad():
        for mod in model.modules():
            if isinstance(mod, nn.Linear):
                b = 1 / math.sqrt(mod.in_features)
                mod.weight.uniform_(-b, b)
        for blk in model.layers:
            blk.attention_norm.weight.uniform_(0.5, 1.5)
            blk.ffn_norm.weight.uniform_(0.5, 1.5)
    model.eval().fuse_w13()
    apply_quantization(model, quant)
    P, T = 9, 12
    prompt = torch.randint(0, 1000, (1, P), device=DEV)
    pos = torch.arange(P, device=DEV)
    model.setup_caches(1, P + T)
    with torch.no_grad():
        model(prompt, pos)
        ref = model(prompt[:, -1:], torch.tensor([P], device=DEV))
        model.setup_caches(1, P + T)
        assert model.enable_fused_kernels()
        model(prompt, pos)
        got = model(prompt[:, -1:], torch.tensor([P], device=DEV))
    assert _rel(got, ref) < 2e-2
    eager, _, _ = generate(model, prompt, T, None)
    dec = GraphDecoder(model, 1, P + T, DEV)
    dec.reset(prompt, prefill(model, prompt, pos))
    dec.capture()
    graphed, _, _ = generate(model, prompt, T, dec)
    assert torch.equal(graphed, eager)


# ---- int8 dynamic activation (tao_int8dq_decode_bf16) ---------------------------------------------
def _int8dq_linear(N, K, seed=0):
    torch.manual_seed(seed)
    lin = nn.Linear(K, N, bias=False, device=DEV, dtype=torch.bfloat16)
    with torch.no_grad():
        lin.weight.uniform_(-1 / math.sqrt(K), 1 / math.sqrt(K))
    quantize_(lin, Int8DynamicActivationInt8WeightConfig())
    from torchao._models.llama.model import _int8dq_parts

    parts = _int8dq_parts(lin)
    assert parts is not None
    return lin, parts


@pytest.mark.parametrize("N,K", [(6144, 4096), (4096, 14336), (128256, 4096), (1000, 512)])
def test_dq_plain_is_the_fused_linear(N, K):
    """No norm, no epilogue: the same kernel and launch shape as int8_dyn_linear (bit-exact)."""
    from torchao._models.llama import kernels

    lin, parts = _int8dq_linear(N, K)
    x = torch.randn(1, 1, K, device=DEV, dtype=torch.bfloat16)
    assert torch.equal(kernels.int8dq_decode(x, *parts), lin(x))


@pytest.mark.parametrize("N,K", [(6144, 4096), (128256, 4096), (2048, 8192)])
def test_dq_rmsnorm_prologue(N, K):
    from torchao._models.llama import kernels

    lin, parts = _int8dq_linear(N, K)
    x = torch.randn(1, 1, K, device=DEV, dtype=torch.bfloat16) * 3
    w = _norm_w(K)
    got = kernels.int8dq_decode(x, *parts, norm_weight=w, eps=1e-5)
    ref = lin(kernels.rmsnorm(x, w, 1e-5))
    # a one-ulp change of a normalised element can move the token's int8 rounding: 1e-2
    assert _rel(got, ref) < 1e-2


@pytest.mark.parametrize("norm", [False, True])
def test_dq_swiglu_and_rope_epilogues(norm):
    from torchao._models.llama import kernels
    from torchao._models.llama.model import ModelArgs, _rope_freqs

    K = 4096
    w = _norm_w(K) if norm else None
    x = torch.randn(1, 1, K, device=DEV, dtype=torch.bfloat16)
    xin = kernels.rmsnorm(x, w, 1e-5) if norm else x
    lin, parts = _int8dq_linear(2 * 1024, K, seed=2)
    got = kernels.int8dq_decode(x, *parts, norm_weight=w, eps=1e-5, epilogue="swiglu")
    ref = kernels.silu_mul(lin(xin))
    if norm:
        assert _rel(got, ref) < 1e-2
    else:
        assert torch.equal(got, ref)
    H, Hkv, D, T, pos = 32, 8, 128, 64, 17
    lin, parts = _int8dq_linear((H + 2 * Hkv) * D, K, seed=3)
    cfg = ModelArgs(n_layer=1, n_head=H, n_local_heads=Hkv, dim=H * D, rope_base=500000)
    freqs = _rope_freqs(cfg, T).to(DEV)
    p = torch.tensor([pos], device=DEV)
    kc = torch.randn(1, Hkv, T, D, device=DEV, dtype=torch.bfloat16)
    vc = torch.randn_like(kc)
    kc_ref, vc_ref = kc.clone(), vc.clone()
    q = kernels.int8dq_decode(x, *parts, norm_weight=w, eps=1e-5, epilogue="rope_kv",
                              rope=(freqs, p, kc, vc, H))
    q_ref = kernels.rope_kv(lin(xin), freqs, p, kc_ref, vc_ref, H)
    for a, b in ((q, q_ref), (kc, kc_ref), (vc, vc_ref)):
        if norm:
            assert _rel(a, b) < 1e-2
        else:
            assert torch.equal(a, b)
