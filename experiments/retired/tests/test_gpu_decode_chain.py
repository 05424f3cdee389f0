"""GPU parity of the persistent int4 decode chain (csrc/decode_chain.hip, torchao.kernel.
decode_chain): every phase's output against the unfused ops computed from the same input
(tao_rmsnorm_bf16 -> tao_int4wo_linear_bf16 with the residual as bias -> tao_silu_mul_bf16), which
the int4 parity tests pin to the oracle; HIP-graph replays (the epoch-counted hand-offs across
launches) give identical outputs every time."""

import math

import pytest
import torch

from oracle import oracle

from torchao._models.llama import kernels
from torchao.kernel.decode_chain import ChainPhase, DecodeChain

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _quant(N, K, g, gen):
    b = 1.0 / math.sqrt(K)
    w = torch.empty(N, K, device=DEV, dtype=torch.bfloat16).uniform_(-b, b, generator=gen)
    return torch.ops.torchao.int4_quantize_pack(w, g, 1e-6)


def _llama_chain(D, qkv, I, V, n_layer, g, seed):
    """A Llama-shaped linears-only chain: per layer wqkv (RMSNorm) -> wo (x = q part, residual =
    layer input) -> w1||w3 (RMSNorm, SwiGLU) -> w2 (residual = h); then the head (RMSNorm)."""
    gen = torch.Generator(device=DEV).manual_seed(seed)
    x0 = torch.randn(D, device=DEV, dtype=torch.bfloat16, generator=gen)
    phases, layer_in, layer_in_phase = [], x0, -1
    for _ in range(n_layer):
        an = torch.empty(D, device=DEV, dtype=torch.bfloat16).uniform_(0.5, 1.5, generator=gen)
        fn = torch.empty(D, device=DEV, dtype=torch.bfloat16).uniform_(0.5, 1.5, generator=gen)
        pq, sq = _quant(qkv, D, g, gen)
        po, so = _quant(D, D, g, gen)
        p13, s13 = _quant(2 * I, D, g, gen)
        p2, s2 = _quant(D, I, g, gen)
        yq = torch.empty(qkv, device=DEV, dtype=torch.bfloat16)
        h = torch.empty(D, device=DEV, dtype=torch.bfloat16)
        gg = torch.empty(I, device=DEV, dtype=torch.bfloat16)
        out = torch.empty(D, device=DEV, dtype=torch.bfloat16)
        base = len(phases)
        phases += [
            ChainPhase(pq, sq, g, x=layer_in, y=yq, x_phase=layer_in_phase, norm_w=an),
            ChainPhase(po, so, g, x=yq, y=h, x_phase=base, residual=layer_in),
            ChainPhase(p13, s13, g, x=h, y=gg, x_phase=base + 1, norm_w=fn, swiglu=True),
            ChainPhase(p2, s2, g, x=gg, y=out, x_phase=base + 2, residual=h),
        ]
        layer_in, layer_in_phase = out, base + 3
    hn = torch.empty(D, device=DEV, dtype=torch.bfloat16).uniform_(0.5, 1.5, generator=gen)
    ph, sh = _quant(V, D, g, gen)
    logits = torch.empty(V, device=DEV, dtype=torch.bfloat16)
    phases.append(ChainPhase(ph, sh, g, x=layer_in, y=logits, x_phase=layer_in_phase, norm_w=hn))
    return phases


def _unfused(p: ChainPhase) -> torch.Tensor:
    """The phase through the per-op kernels, from the chain's own input buffer."""
    K = p.packed.shape[1] * 8
    x = p.x[:K].reshape(1, K)
    if p.norm_w is not None:
        x = kernels.rmsnorm(x.contiguous(), p.norm_w, p.eps)
    bias = None if p.swiglu else p.residual
    y = torch.ops.torchao.int4_weight_only_linear(x.contiguous(), p.packed, p.scale_and_zero,
                                                  p.group_size, bias)
    if p.swiglu:
        y = kernels.silu_mul(y.contiguous())
        if p.residual is not None:
            y = y + p.residual
    return y.reshape(-1)


def _check_phases(phases):
    for i, p in enumerate(phases):
        got = p.y[: (p.packed.shape[0] // 2 if p.swiglu else p.packed.shape[0])].float()
        ref = _unfused(p).float()
        # same bf16 roundings; only the fp32 sum order of each row differs (launch shape)
        ulp = ref.abs().clamp_min(ref.abs().max() * 2 ** -8) * 2 ** -7
        bad = (got - ref).abs() > 2 * ulp
        assert not bool(bad.any()), (i, int(bad.sum()), float((got - ref).abs().max()))


@pytest.mark.parametrize("g", [32, 128])
def test_chain_small_llama_matches_unfused_ops(g):
    phases = _llama_chain(D=512, qkv=768, I=1024, V=1000, n_layer=2, g=g, seed=1)
    chain = DecodeChain(phases)
    chain.run()
    torch.cuda.synchronize()
    chain.check()
    _check_phases(phases)
    # one-token oracle check of the first linear (the CPU dequant path)
    p = phases[1]  # wo: plain linear + residual
    q, s, z = (t.cpu() for t in _plain(p))
    x = p.x[:512].reshape(1, 512).cpu()
    ref = oracle.int4_linear(x, q, s, z, g, p.residual.cpu())
    assert oracle.rel_l2(p.y.reshape(1, -1).cpu(), ref) < 1e-2


def _plain(p: ChainPhase):
    qq = torch.ops.torchao.int4_unpack(p.packed)
    return qq, p.scale_and_zero[..., 0].contiguous(), p.scale_and_zero[..., 1].contiguous()


def test_chain_graph_replays_identical_and_counts_epochs():
    phases = _llama_chain(D=1024, qkv=1536, I=2048, V=2048, n_layer=3, g=32, seed=2)
    chain = DecodeChain(phases)
    stream = torch.cuda.Stream()
    stream.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(stream):
        chain.run()  # eager
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=stream):
            chain.run()
    torch.cuda.current_stream().wait_stream(stream)
    torch.cuda.synchronize()
    first = [p.y.clone() for p in phases]
    for _ in range(5):
        for p in phases:
            p.y.zero_()
        graph.replay()
        torch.cuda.synchronize()
        for p, f in zip(phases, first):
            assert torch.equal(p.y, f)
    aborted, launches = chain.status()
    assert aborted is None and launches == 6  # eager + 5 replays (capture does not run)
    _check_phases(phases)


def test_chain_llama3_8b_full_width():
    """Llama-3-8B shapes (wqkv 6144x4096, wo 4096^2, w1||w3 28672x4096, w2 4096x14336, head
    128256x4096), two layers + head."""
    phases = _llama_chain(D=4096, qkv=6144, I=14336, V=128256, n_layer=2, g=32, seed=3)
    chain = DecodeChain(phases)
    for _ in range(3):
        chain.run()
    torch.cuda.synchronize()
    chain.check()
    _check_phases(phases)
