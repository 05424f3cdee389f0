"""RMSNorm -> int4 wqkv -> RoPE + KV write -> decode attention in one launch
(tao_int4wo_qkv_attn_bf16) against the two launches it replaces: the fused wqkv GEMV
(tao_int4wo_decode_bf16, epilogue rope_kv) then the one-pass decode attention. The GEMV part runs
the same launch shape and arithmetic, so q and the caches are bit-identical; the attention walks
the keys in another order (split ranges of 4 waves instead of 16 waves over all keys), so its
output is held to the one-pass kernel's bar against fp32 attention (2e-2) and to a few bf16 ulps
of the one-pass output."""

import math

import pytest
import torch
import torch.nn as nn

from torchao.quantization import Int4WeightOnlyConfig, quantize_

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _setup(H, Hkv, K, T, g=32, seed=0):
    from torchao._models.llama.model import ModelArgs, _int4_parts, _rope_freqs

    D = 128
    N = (H + 2 * Hkv) * D
    torch.manual_seed(seed)
    lin = nn.Linear(K, N, bias=False, device=DEV, dtype=torch.bfloat16)
    with torch.no_grad():
        lin.weight.uniform_(-1 / math.sqrt(K), 1 / math.sqrt(K))
    quantize_(lin, Int4WeightOnlyConfig(group_size=g))
    parts = _int4_parts(lin)
    cfg = ModelArgs(n_layer=1, n_head=H, n_local_heads=Hkv, dim=H * D, rope_base=500000)
    freqs = _rope_freqs(cfg, T).to(DEV)
    gen = torch.Generator(device=DEV).manual_seed(seed + 1)
    w = (torch.rand(K, device=DEV, generator=gen) + 0.5).to(torch.bfloat16)
    kc = torch.randn(1, Hkv, T, D, device=DEV, dtype=torch.bfloat16, generator=gen)
    vc = torch.randn(1, Hkv, T, D, device=DEV, dtype=torch.bfloat16, generator=gen)
    x = torch.randn(1, 1, K, device=DEV, dtype=torch.bfloat16, generator=gen)
    return parts, freqs, w, kc, vc, x


def _attn_fp32(q, kc, vc, p, scale):
    """q [1, H, 1, D] over keys 0..p of the caches [1, Hkv, T, D] -> [1, 1, H * D] fp32."""
    H, Hkv = q.shape[1], kc.shape[1]
    k = kc[0, :, : p + 1].float().repeat_interleave(H // Hkv, 0)  # [H, L, D]
    v = vc[0, :, : p + 1].float().repeat_interleave(H // Hkv, 0)
    s = torch.einsum("hd,hld->hl", q[0, :, 0].float(), k) * scale
    return torch.einsum("hl,hld->hd", torch.softmax(s, -1), v).reshape(1, 1, -1)


@pytest.mark.parametrize("splits", [1, 2, 4])
@pytest.mark.parametrize("H,Hkv,K,T,g", [(32, 8, 4096, 328, 32), (8, 2, 1024, 200, 64),
                                         (4, 4, 512, 64, 32), (16, 2, 8192, 1100, 128)])
def test_qkv_attn_matches_two_launches(H, Hkv, K, T, g, splits):
    from torchao._models.llama import kernels

    parts, freqs, w, kc, vc, x = _setup(H, Hkv, K, T, g)
    N = parts[0].shape[0]
    assert kernels.qkv_attn_supported(N, K, H, Hkv, 128)
    scale = 1 / math.sqrt(128)
    # positions across the 16-key steps and the split boundaries (empty trailing splits at 0-17)
    for pos in sorted({0, 1, 15, 16, 17, 63, T // 2, T - 2, T - 1}):
        p = torch.tensor([pos], device=DEV)
        kr, vr = kc.clone(), vc.clone()
        q_ref = kernels.int4_decode(x, *parts, norm_weight=w, eps=1e-5, epilogue="rope_kv",
                                    rope=(freqs, p, kr, vr, H))
        one_pass = kernels.attn_decode(q_ref, kr, vr, p, scale)
        kg, vg = kc.clone(), vc.clone()
        got = kernels.int4_qkv_attn(x, *parts, w, 1e-5, freqs, p, kg, vg, H, scale, splits)
        torch.cuda.synchronize()
        assert torch.equal(kg, kr) and torch.equal(vg, vr), pos  # the GEMV part bit for bit
        ref = _attn_fp32(q_ref, kr, vr, pos, scale)
        torch.testing.assert_close(got.float(), ref, rtol=2e-2, atol=2e-2)
        torch.testing.assert_close(got.float(), one_pass.float(), rtol=2e-2, atol=2e-2)
        rel = float((got.float() - one_pass.float()).norm() / one_pass.float().norm())
        assert rel < 4e-3, (pos, rel)
    kernels.check_decode_status()  # no position error, no ticket timeout


def test_qkv_attn_graph_replay_and_tickets():
    """Captured once, replayed at advancing positions read at replay time: equal to eager calls;
    a long run of launches (tickets must return to zero after every one) stays equal; a position
    past the cache writes no row and sets status bit 1; unsupported shapes are refused."""
    from torchao import _lib
    from torchao._models.llama import kernels

    H, Hkv, K, T = 32, 8, 4096, 96
    parts, freqs, w, kc, vc, x = _setup(H, Hkv, K, T, seed=5)
    scale = 1 / math.sqrt(128)
    kernels.check_decode_status()
    # eager reference over positions 40..71 on its own caches
    ke, ve = kc.clone(), vc.clone()
    eager = []
    for pos in range(40, 72):
        eager.append(kernels.int4_qkv_attn(x, *parts, w, 1e-5, freqs,
                                           torch.tensor([pos], device=DEV), ke, ve, H, scale))
    # graph: one capture, the position tensor advanced between replays
    kg, vg = kc.clone(), vc.clone()
    p = torch.tensor([40], device=DEV)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            out = kernels.int4_qkv_attn(x, *parts, w, 1e-5, freqs, p, kg, vg, H, scale)
    torch.cuda.current_stream().wait_stream(s)
    for i, pos in enumerate(range(40, 72)):
        p.fill_(pos)
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(out, eager[i]), pos
    assert torch.equal(kg, ke) and torch.equal(vg, ve)
    # many launches back to back on one stream: each must start from zeroed tickets
    outs = [kernels.int4_qkv_attn(x, *parts, w, 1e-5, freqs, torch.tensor([50], device=DEV),
                                  kg, vg, H, scale) for _ in range(64)]
    for o in outs:
        assert torch.equal(o, outs[0])
    kernels.check_decode_status()
    # a position past the cache: no row written, reported; the call itself completes
    before = (kg.clone(), vg.clone())
    bad = kernels.int4_qkv_attn(x, *parts, w, 1e-5, freqs, torch.tensor([T], device=DEV), kg, vg,
                                H, scale)
    torch.cuda.synchronize()
    assert torch.equal(kg, before[0]) and torch.equal(vg, before[1])
    assert bool(torch.isfinite(bad.float()).all())
    with pytest.raises(RuntimeError, match="past the KV cache"):
        kernels.check_decode_status()
    kernels.check_decode_status()
    # refused shapes
    assert not kernels.qkv_attn_supported(6144, 4096, 32, 8, 64)
    assert not kernels.qkv_attn_supported(28672, 4096, 32, 8, 128)
    with pytest.raises(RuntimeError, match="splits"):
        kernels.int4_qkv_attn(x, *parts, w, 1e-5, freqs, p, kg, vg, H, scale, 3)
    assert _lib.lib().tao_int4wo_qkv_attn_supported(6144, 4096, 32, 8, 128) == 1
