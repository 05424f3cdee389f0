"""Seeded random-shape parity sweep of the three linears against the oracle (GPU).

Shapes are drawn (fixed seeds) over M 1..300, N 8..3000 (multiples of 8), K multiples of the group
size up to 3072, every group size, with and without bias, so the launch-shape heuristics, the
measured shape table's buckets, the split-K / k-group combinations and every GEMV tail case get
exercised off the Llama grid. Each case also runs on the 32x32x16 int4 kernel and with the shape
table off, and the three results must agree within the oracle bars.
"""

import random

import pytest
import torch

from oracle import oracle

from torchao import _lib

pytestmark = pytest.mark.gpu
DEV = "cuda"
TOL_REF = 1e-2
TOL_FP32 = 4e-3


def _cases(n, seed):
    rng = random.Random(seed)
    out = []
    for _ in range(n):
        g = rng.choice([32, 64, 128, 256])
        M = rng.choice([1, 2, 3, 4, 5, 7, 16, 33, 64, 100, 128, 129, 257, 300])
        N = 8 * rng.randint(1, 375)
        K = g * rng.randint(1, 3072 // g)
        out.append((M, N, K, g, rng.random() < 0.5))
    return out


@pytest.mark.parametrize("M,N,K,g,with_bias", _cases(24, seed=2026))
def test_int4_random_shapes(M, N, K, g, with_bias):
    w = oracle.make_linear_weight(N, K, seed=N * 7 + K)
    s, z = oracle.int4_qparams(w, g)
    q = oracle.int4_quantize(w, s, z, g)
    x = oracle.make_activation(M, K, seed=M + N)
    bias = oracle.make_activation(1, N, seed=K).reshape(N) if with_bias else None
    packed = torch.ops.torchao.int4_pack(q.to(DEV))
    sz = torch.stack([s, z], dim=-1).contiguous().to(DEV)
    xd = x.to(DEV)
    bd = bias.to(DEV) if bias is not None else None
    ref32 = oracle.int4_linear_fp32(x, q, s, z, g, bias)
    y = torch.ops.torchao.int4_weight_only_linear(xd, packed, sz, g, bd).cpu()
    assert oracle.rel_l2(y, ref32) < TOL_FP32
    assert oracle.rel_l2(y, oracle.int4_linear(x, q, s, z, g, bias)) < TOL_REF
    outs = []
    try:
        _lib.call("tao_tune_gemm_table", 1)
        outs.append(torch.ops.torchao.int4_weight_only_linear(xd, packed, sz, g, bd).cpu())
        _lib.call("tao_tune_gemm_table", 0)
        if M > 4:  # MFMA path: the 32x32x16 kernel at its own shape
            _lib.call("tao_tune_int4_mfma32", 1)
            outs.append(torch.ops.torchao.int4_weight_only_linear(xd, packed, sz, g, bd).cpu())
    finally:
        _lib.call("tao_tune_reset")
    for o in outs:
        assert oracle.rel_l2(o, ref32) < TOL_FP32


@pytest.mark.parametrize("M,N,K,g,with_bias", _cases(16, seed=7))
def test_int8_random_shapes(M, N, K, g, with_bias):
    w = oracle.make_linear_weight(N, K, seed=N + 3 * K)
    x = oracle.make_activation(M, K, seed=M * 5 + N)
    bias = oracle.make_activation(1, N, seed=N).reshape(N) if with_bias else None
    xd = x.to(DEV)
    bd = bias.to(DEV) if bias is not None else None
    s8 = oracle.int8_weight_qparams(w)
    q8 = oracle.int8_weight_quantize(w, s8)
    y8 = torch.ops.torchao.int8_weight_only_linear(xd, q8.to(DEV), s8.to(DEV), bd).cpu()
    assert oracle.rel_l2(y8, oracle.int8wo_linear(x, q8, s8, bias)) < TOL_REF
    wq, ws = oracle.int8_dyn_weight(w)
    xq, xs = oracle.int8_act_quant(x)
    ref = oracle.int8_scaled_mm(xq, xs, wq, ws, bias, epilogue="cpu")
    yd = torch.ops.torchao.int8_scaled_mm(xq.to(DEV), xs.to(DEV), wq.to(DEV), ws.to(DEV), bd)
    assert torch.equal(yd.cpu(), ref)  # exact integer accumulation, reference epilogue order
    try:
        _lib.call("tao_tune_gemm_table", 1)
        yh = torch.ops.torchao.int8_scaled_mm(xq.to(DEV), xs.to(DEV), wq.to(DEV), ws.to(DEV), bd)
    finally:
        _lib.call("tao_tune_reset")
    assert torch.equal(yh.cpu(), ref)
