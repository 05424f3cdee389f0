"""The C++ dispatcher kernels of the per-linear ops (csrc/torch_ops.cpp) against the Python impls
they replace (torchao/ops.py, still defined): same C-ABI kernels, so outputs must be
bit-identical; same argument checks and messages; capturable in a HIP graph."""

import pytest
import torch

from torchao import ops

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _int4_weight(N, K, g, seed=0):
    gen = torch.Generator().manual_seed(seed)
    q = torch.randint(0, 16, (N, K), generator=gen, dtype=torch.int32)
    packed = torch.ops.torchao.int4_pack(q.to(DEV))
    s = (torch.rand(N, K // g, generator=gen) * 0.02 + 0.001).to(torch.bfloat16)
    z = (torch.randn(N, K // g, generator=gen) * 0.05).to(torch.bfloat16)
    return packed, torch.stack([s, z], -1).contiguous().to(DEV)


def _int8_weight(N, K, seed=0):
    gen = torch.Generator().manual_seed(seed)
    w = torch.randint(-128, 128, (N, K), generator=gen, dtype=torch.int8)
    s = (torch.rand(N, generator=gen) * 0.01 + 1e-3).to(torch.bfloat16)
    return w.to(DEV), s.to(DEV)


def test_native_kernels_loaded():
    assert "int4_weight_only_linear" in ops.native_dispatch(), ops._native_error


@pytest.mark.parametrize("M", [1, 3, 64])
@pytest.mark.parametrize("bias", [False, True])
def test_int4_cpp_matches_python_impl(M, bias):
    N, K, g = 256, 1024, 32
    packed, sz = _int4_weight(N, K, g)
    x = torch.randn(2, M, K, device=DEV, dtype=torch.bfloat16)
    b = torch.randn(N, device=DEV, dtype=torch.bfloat16) if bias else None
    y = torch.ops.torchao.int4_weight_only_linear(x, packed, sz, g, b)
    y_py = ops._int4_linear_cuda(x, packed, sz, g, b)
    assert y.shape == (2, M, N) and torch.equal(y, y_py)


@pytest.mark.parametrize("M", [1, 5, 128])
def test_int8_cpp_matches_python_impl(M):
    N, K = 256, 512
    w, s = _int8_weight(N, K)
    x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    b = torch.randn(N, device=DEV, dtype=torch.bfloat16)
    assert torch.equal(torch.ops.torchao.int8_weight_only_linear(x, w, s, b),
                       ops._int8wo_linear_cuda(x, w, s, b))
    q, xs = torch.ops.torchao.int8_quantize_per_token(x)
    q_py, xs_py = ops._int8_quant_cuda(x)
    assert torch.equal(q, q_py) and torch.equal(xs, xs_py) and xs.shape == (M, 1)
    assert torch.equal(torch.ops.torchao.int8_scaled_mm(q, xs, w, s, b),
                       ops._int8_scaled_mm_cuda(q, xs, w, s, b))
    if M == 1:
        assert torch.equal(torch.ops.torchao.int8_dyn_linear(x, w, s, b),
                           ops._int8_dyn_linear_cuda(x, w, s, b))


def test_cpp_argument_checks():
    packed, sz = _int4_weight(64, 256, 32)
    x = torch.randn(1, 256, device=DEV, dtype=torch.bfloat16)
    with pytest.raises(RuntimeError, match="qGroupSize must be 32, 64, 128, or 256"):
        torch.ops.torchao.int4_weight_only_linear(x, packed, sz, 48)
    with pytest.raises(RuntimeError, match="scales_and_zeros must be"):
        torch.ops.torchao.int4_weight_only_linear(x, packed, sz[:, :4], 32)
    with pytest.raises(RuntimeError, match="needs bf16 input"):
        torch.ops.torchao.int4_weight_only_linear(x.float(), packed, sz, 32)
    with pytest.raises(RuntimeError, match="x last dim"):
        torch.ops.torchao.int4_weight_only_linear(x[:, :128], packed, sz, 32)
    w, s = _int8_weight(64, 256)
    with pytest.raises(RuntimeError, match="one token"):
        torch.ops.torchao.int8_dyn_linear(torch.randn(2, 256, device=DEV, dtype=torch.bfloat16),
                                          w, s)
    with pytest.raises(RuntimeError, match="scale must have N elements"):
        torch.ops.torchao.int8_weight_only_linear(x, w, s[:3])


def test_cpp_kernel_status_surfaces_as_runtime_error():
    # a K that is not a multiple of 32 passes the schema checks but not the C-ABI's (K % g)
    w, s = _int8_weight(64, 100)
    x = torch.randn(1, 100, device=DEV, dtype=torch.bfloat16)
    try:
        ops._int8_dyn_linear_cuda(x, w, s)
    except RuntimeError as e:
        py_msg = str(e)
        with pytest.raises(RuntimeError, match="tao_int8_dyn_linear_bf16 failed"):
            torch.ops.torchao.int8_dyn_linear(x, w, s)
        assert "tao_int8_dyn_linear_bf16 failed" in py_msg
    else:  # the kernel accepts this K: both paths must agree
        assert torch.equal(torch.ops.torchao.int8_dyn_linear(x, w, s),
                           ops._int8_dyn_linear_cuda(x, w, s))


def test_cpp_ops_capture_in_graph():
    N, K, g = 512, 1024, 64
    packed, sz = _int4_weight(N, K, g, seed=3)
    x = torch.randn(1, K, device=DEV, dtype=torch.bfloat16)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        torch.ops.torchao.int4_weight_only_linear(x, packed, sz, g)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=s):
            y = torch.ops.torchao.int4_weight_only_linear(x, packed, sz, g)
    torch.cuda.current_stream().wait_stream(s)
    x.copy_(torch.randn_like(x))
    graph.replay()
    torch.cuda.synchronize()
    assert torch.equal(y, ops._int4_linear_cuda(x, packed, sz, g))
