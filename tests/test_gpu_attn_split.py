"""Split decode attention (tao_attn_decode_split_bf16) and its two finishers: the merge kernel
(tao_attn_merge_bf16) and the int4 wo linear with the merge as its x prologue
(tao_int4wo_attn_out_bf16). Together they replace the one-pass decode attention + wo (+ residual)
of the gpt-fast harness at decode (reference torchao/_models/llama/model.py:462-474 and the wo
linear after it).

Bars: the merged attention against fp32 SDPA over keys 0..L-1 (the one-pass kernel's bar,
rtol / atol 2e-2) and within one bf16 rounding of the one-pass kernel (same fp32 math, other
summation order); the fused wo bit-identical to merge -> the same GEMV launch shape with x
staged in LDS (tao_tune_int4_xlds 1) -> + residual; run-to-run identical; graph-capturable."""

import math

import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from torchao.quantization import Int4WeightOnlyConfig, quantize_

pytestmark = pytest.mark.gpu

DEV = "cuda"
D = 128


def _kv(B, Hkv, T, H, seed=0):
    g = torch.Generator(device=DEV).manual_seed(seed)
    kc = torch.randn(B, Hkv, T, D, device=DEV, dtype=torch.bfloat16, generator=g)
    vc = torch.randn(B, Hkv, T, D, device=DEV, dtype=torch.bfloat16, generator=g)
    q = torch.randn(B, H, 1, D, device=DEV, dtype=torch.bfloat16, generator=g)
    return q, kc, vc


@pytest.mark.parametrize("splits", [2, 4])
@pytest.mark.parametrize("G", [1, 4, 8])
def test_split_merge_matches_sdpa_and_one_pass(splits, G):
    from torchao._models.llama import kernels

    Hkv = 8 // G if G < 8 else 2
    H = Hkv * G
    # lengths across the 16-key rounding of the ranges, empty trailing splits (L = 1, 15, 17 at
    # 4 splits), one and two 256-key rounds per split, the full cache
    for T, L in ((64, 1), (64, 15), (64, 17), (64, 33), (64, 64), (328, 129), (328, 328),
                 (1024, 700), (1024, 1024)):
        q, kc, vc = _kv(2, Hkv, T, H, seed=L)
        pos = torch.tensor([L - 1], device=DEV)
        scale = 1 / math.sqrt(D)
        part = kernels.attn_decode_split(q, kc, vc, pos, scale, splits)
        got = kernels.attn_merge(part, 2, H)
        again = kernels.attn_merge(kernels.attn_decode_split(q, kc, vc, pos, scale, splits), 2, H)
        assert torch.equal(got, again)
        ref = F.scaled_dot_product_attention(q.float(), kc[:, :, :L].float(),
                                             vc[:, :, :L].float(), enable_gqa=True)
        ref = ref.transpose(1, 2).reshape(2, 1, H * D)
        torch.testing.assert_close(got.float(), ref, rtol=2e-2, atol=2e-2)
        one = kernels.attn_decode(q, kc, vc, pos, scale)
        # same fp32 softmax and P.V, another association of the sums: one bf16 rounding apart
        diff = (got.float() - one.float()).abs()
        assert (diff <= one.float().abs() * 2 ** -7 + 1e-6).all(), diff.max()
        # an empty split's record: m = -inf, l = 0, o = 0
        C = ((L + splits - 1) // splits + 15) // 16 * 16
        for s in range(splits):
            rec = part[:, s]
            if s * C >= L:
                assert torch.isinf(rec[:, 128]).all() and (rec[:, 129] == 0).all()
                assert (rec[:, :128] == 0).all()
            else:
                assert torch.isfinite(rec[:, 128]).all() and (rec[:, 129] >= 1).all()


def _int4_wo(N, K, g=32, seed=0):
    torch.manual_seed(seed)
    lin = nn.Linear(K, N, bias=False, device=DEV, dtype=torch.bfloat16)
    with torch.no_grad():
        lin.weight.uniform_(-1 / math.sqrt(K), 1 / math.sqrt(K))
    quantize_(lin, Int4WeightOnlyConfig(group_size=g))
    from torchao._models.llama.model import _int4_parts

    return lin, _int4_parts(lin)


@pytest.mark.parametrize("H,N,g,splits", [(32, 4096, 32, 2), (32, 4096, 32, 4),
                                          (64, 8192, 32, 2), (8, 1024, 128, 2),
                                          (32, 1000, 64, 4)])
def test_int4_attn_out_is_merge_then_linear(H, N, g, splits):
    from torchao._models.llama import kernels
    from torchao.kernel.tuning import tuning

    K = H * D
    lin, parts = _int4_wo(N, K, g)
    Hkv = max(H // 4, 1)
    q, kc, vc = _kv(1, Hkv, 512, H, seed=H + N)
    pos = torch.tensor([300], device=DEV)
    part = kernels.attn_decode_split(q, kc, vc, pos, 1 / math.sqrt(D), splits)
    res = torch.randn(1, 1, N, device=DEV, dtype=torch.bfloat16)
    got = kernels.int4_attn_out(part, H, *parts, residual=res)
    assert torch.equal(got, kernels.int4_attn_out(part, H, *parts, residual=res))
    x = kernels.attn_merge(part, 1, H)
    with tuning(int4_xlds=1):  # the same launch shape, x staged raw in LDS
        y = lin(x)
    assert torch.equal(got, y + res), (got.float() - (y + res).float()).abs().max()
    # without a residual: the plain linear of the merged x
    got0 = kernels.int4_attn_out(part, H, *parts)
    assert torch.equal(got0, y)
    # against the built-in GEMV shape of the plain linear: other sum order, within the bars
    ref = lin(x) + res
    err = (got.float() - ref.float()).norm() / ref.float().norm()
    assert err < 4e-3, err


def test_attn_split_pair_graph_capture_and_errors():
    from torchao import _lib
    from torchao._models.llama import kernels

    H, N, splits = 32, 4096, 2
    lin, parts = _int4_wo(N, H * D)
    q, kc, vc = _kv(1, 8, 256, H)
    pos = torch.tensor([100], device=DEV)
    res = torch.randn(1, 1, N, device=DEV, dtype=torch.bfloat16)

    def step():
        part = kernels.attn_decode_split(q, kc, vc, pos, 1 / math.sqrt(D), splits)
        return kernels.int4_attn_out(part, H, *parts, residual=res)

    eager = step()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        step()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            out = step()
    torch.cuda.current_stream().wait_stream(s)
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(out, eager)
    pos.fill_(200)  # the graph reads the position at replay: a longer prefix
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(out, step())
    assert not torch.equal(out, eager)

    part = kernels.attn_decode_split(q, kc, vc, pos, 1 / math.sqrt(D), 2)
    with pytest.raises(RuntimeError, match="splits must be 2 or 4"):
        _lib.call("tao_attn_decode_split_bf16", q.data_ptr(), kc.data_ptr(), vc.data_ptr(),
                  pos.data_ptr(), part.data_ptr(), 1, H, 8, D, 256, 0.1, 3, None)
    with pytest.raises(RuntimeError, match="n_head \\* 128"):
        _lib.call("tao_int4wo_attn_out_bf16", part.data_ptr(), 2, H - 1, parts[0].data_ptr(),
                  parts[1].data_ptr(), N, H * D, 32, None, res.data_ptr(), None)
