"""The persistent LDS-DMA decode FFN engine (tao_int4wo_ffn_engine_bf16, csrc/decode_engine.hip)
against the two fused launches it replaces (tao_int4wo_decode_bf16 RMSNorm + w1||w3 + SwiGLU,
then the w2 GEMV with the residual as bias) and against the fp32 oracle of the same int4 weights.

Each stage is checked at its own scale (the microarch guide's rule for fused stages): the
SwiGLU outputs the engine publishes (stage 1) against the launch path's SwiGLU output, and the
block output (stage 2). The engine sums each row in another order than the GEMV launches (one
wave per row chunk, three consumer waves per w2 row), so the bar is the re-association one:
rel L2 <= 4e-3 against the launch path, <= 1e-2 against the fp32 oracle (north star), and
run-to-run / graph-replay bit identity (fixed summation order)."""

import math

import pytest
import torch
import torch.nn as nn

from torchao.quantization import Int4WeightOnlyConfig, quantize_

pytestmark = pytest.mark.gpu
DEV = "cuda"
DIM, INTER, G = 4096, 14336, 32


def _lin(N, K, seed):
    torch.manual_seed(seed)
    lin = nn.Linear(K, N, bias=False, device=DEV, dtype=torch.bfloat16)
    with torch.no_grad():
        lin.weight.uniform_(-1 / math.sqrt(K), 1 / math.sqrt(K))
    quantize_(lin, Int4WeightOnlyConfig(group_size=G))
    from torchao._models.llama.model import _int4_parts

    return lin, _int4_parts(lin)


def _rel(a, b):
    a, b = a.float().flatten(), b.float().flatten()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


@pytest.fixture(scope="module")
def ffn():
    from torchao._models.llama import kernels

    if not kernels.ffn_engine_supported(DIM, INTER, G):
        pytest.skip("ffn engine: device / shape unsupported")
    w13, p13 = _lin(2 * INTER, DIM, 1)   # rows interleaved (w1_i, w3_i) as FeedForward.fuse_w13
    w2, p2 = _lin(DIM, INTER, 2)
    gen = torch.Generator(device=DEV).manual_seed(3)
    nw = (torch.rand(DIM, device=DEV, generator=gen) + 0.5).to(torch.bfloat16)
    return w13, p13, w2, p2, nw


def _launch_path(h, nw, p13, p2):
    """the two fused launches of FeedForward.forward_fused (model.py)"""
    from torchao import _lib
    from torchao._models.llama import kernels

    g = kernels.int4_decode(h, *p13, norm_weight=nw, eps=1e-5, epilogue="swiglu")
    out = torch.empty_like(h)
    _lib.call("tao_int4wo_linear_bf16", g.data_ptr(), p2[0].data_ptr(), p2[1].data_ptr(),
              h.data_ptr(), out.data_ptr(), 1, DIM, INTER, G,
              torch.cuda.current_stream().cuda_stream)
    return g, out


def _payload(h):
    from torchao._models.llama import kernels

    ws = kernels.ffn_engine_workspace(h.device)
    return ws[1024:1024 + INTER // 2].view(torch.bfloat16).reshape(-1)  # 4 KiB in: [I/2] u32


def _shards(h):
    from torchao._models.llama import kernels

    ws = kernels.ffn_engine_workspace(h.device)
    return [int(ws[64 + 32 * s].item()) for s in range(8)]


@pytest.mark.parametrize("scale", [1.0, 8.0])
def test_engine_matches_launch_path_and_oracle(ffn, scale):
    from torchao._models.llama import kernels

    w13, p13, w2, p2, nw = ffn
    gen = torch.Generator(device=DEV).manual_seed(int(scale * 10))
    h = (torch.randn(1, 1, DIM, device=DEV, generator=gen) * scale).to(torch.bfloat16)
    g_ref, out_ref = _launch_path(h, nw, p13, p2)
    epoch = int(kernels.ffn_engine_workspace(h.device)[0].item())
    out = kernels.int4_ffn_engine(h, nw, 1e-5, p13, p2)
    torch.cuda.synchronize()
    # stage 1: the SwiGLU output as published, and every workgroup's arrival counted (32 per
    # shard counter per launch: the counters reach 32 x epoch)
    assert _shards(h) == [32 * epoch] * 8
    assert _rel(_payload(h), g_ref) < 4e-3
    assert int(kernels.ffn_engine_workspace(h.device)[0].item()) == epoch + 1
    # stage 2: the block output
    assert _rel(out - h, out_ref - h) < 4e-3
    # against the fp32 oracle of the same int4 weights
    wd13 = w13.weight.dequantize().float()
    wd2 = w2.weight.dequantize().float()
    hf = h.float().reshape(-1)
    xn = hf * torch.rsqrt(hf.pow(2).mean() + 1e-5) * nw.float()
    ab = (wd13 @ xn).reshape(-1, 2)
    sg = torch.nn.functional.silu(ab[:, 0]) * ab[:, 1]
    ref = hf + wd2 @ sg
    # the block output against fp32 (bf16 output rounding included), and no worse than the
    # launch path's own distance from it
    e_eng, e_lp = _rel(out.float().reshape(-1), ref), _rel(out_ref.float().reshape(-1), ref)
    assert e_eng < 1e-2 and e_eng <= 1.25 * e_lp + 1e-3, (e_eng, e_lp)
    # the FFN branch alone (before the residual's rounding): same bar for both paths
    ffn = wd2 @ sg
    assert _rel(out.float().reshape(-1) - hf, ffn) <= 1.25 * _rel(out_ref.float().reshape(-1) - hf,
                                                                  ffn) + 1e-3
    kernels.check_decode_status()


def test_engine_deterministic_and_graph_replay(ffn):
    from torchao._models.llama import kernels

    _, p13, _, p2, nw = ffn
    h = torch.randn(1, 1, DIM, device=DEV, dtype=torch.bfloat16)
    first = kernels.int4_ffn_engine(h, nw, 1e-5, p13, p2)
    for _ in range(5):
        assert torch.equal(kernels.int4_ffn_engine(h, nw, 1e-5, p13, p2), first)
    # a chain of 4 dependent blocks captured once, replayed 3 times with new inputs
    x_in = h.clone()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=s):
            y = x_in
            for _ in range(4):
                y = kernels.int4_ffn_engine(y, nw, 1e-5, p13, p2)
            y_out = y
    torch.cuda.current_stream().wait_stream(s)
    for rep in range(3):
        x_in.copy_(torch.randn(1, 1, DIM, device=DEV, dtype=torch.bfloat16) * (1 + rep))
        e = x_in.clone()
        for _ in range(4):
            e = kernels.int4_ffn_engine(e, nw, 1e-5, p13, p2)
        graph.replay()
        torch.cuda.synchronize()
        assert torch.equal(y_out, e), rep
    kernels.check_decode_status()


def test_engine_rejects_bad_arguments(ffn):
    from torchao._models.llama import kernels

    _, p13, _, p2, nw = ffn
    assert not kernels.ffn_engine_supported(8192, 28672, 32)
    assert not kernels.ffn_engine_supported(4096, 14336, 64)
    h = torch.randn(1, 1, DIM, device=DEV, dtype=torch.bfloat16)
    with pytest.raises(RuntimeError):
        kernels.int4_ffn_engine(h, nw, 1e-5, p2, p13)  # swapped linears: shape check
