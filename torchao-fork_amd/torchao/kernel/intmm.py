"""int8 matmul entry points (reference torchao/kernel/intmm.py:30-143).

``safe_int_mm(a, b)`` = int8 [M, K] @ int8 [K, N] -> exact int32 [M, N], with the reference's
routing (:30-88): the same-device assert; a host int32 matmul for CPU operands and for shapes the
BLAS path rejects (K or N not a non-zero multiple of 8); otherwise ``torch._int_mm`` (hipBLASLt
on ROCm), and where that rejects a shape (small M on some builds) an fp64 matmul on the device,
which is exact here: every product is below 2^14 and every partial sum below 2^53, so the result
does not depend on the summation order. (The reference falls back to fp32, exact only while
|sum| < 2^24, i.e. not for K = 4096 at full int8 range.)

``int_scaled_matmul(a, b, scales1)`` = ``(a @ b) * scales1`` (:108-143). On the GPU with bf16
row scales and a ``b`` that is the transpose of a contiguous [N, K] weight (the shape every int8
linear produces) it runs the gfx950 int8-MFMA kernel with the row scale fused into its epilogue,
bit-identical to the reference's ``c.to(bf16) * scales`` (the int32 result is cast to the
scale's dtype before the multiply on both devices). The Triton autotuner path of the reference
(``TORCHAO_AUTOTUNER_ENABLE``) does not exist here.
"""

import torch

__all__ = ["safe_int_mm", "int_scaled_matmul"]


def _is_compiling(t: torch.Tensor) -> bool:
    return torch.compiler.is_compiling() or "FakeTensor" in type(t).__name__


def safe_int_mm(input: torch.Tensor, mat2: torch.Tensor) -> torch.Tensor:
    """int8 [M, K] @ int8 [K, N] -> int32 [M, N], exact."""
    assert input.dtype == torch.int8 and mat2.dtype == torch.int8
    if _is_compiling(input):  # reference :46-52
        from torch._higher_order_ops.out_dtype import out_dtype

        if input.device.type == "cpu":
            return out_dtype(torch.ops.aten.mm.default, torch.int32, input.float(), mat2.float())
        return out_dtype(torch.ops.aten.mm.default, torch.int32, input, mat2)
    assert mat2.device == input.device, (
        f"need both tensors to be on the same device but got {mat2.device} and {input.device}"
    )
    K, N = mat2.shape
    bad_dims = not (K % 8 == 0 and K > 0 and N % 8 == 0 and N > 0)
    if input.device.type == "cpu" or bad_dims:  # reference :58-70
        return torch.matmul(input.cpu().to(torch.int32), mat2.cpu().to(torch.int32)).to(
            input.device)
    if not mat2.is_contiguous():  # reference :73-80
        mat2 = mat2.contiguous()
    if not input.is_contiguous() and input.shape[0] % 8 != 0:
        input = input.contiguous()
    try:
        return torch._int_mm(input, mat2)
    except RuntimeError:
        # exact on the device (see the module docstring), instead of the reference's fp32
        return torch.matmul(input.to(torch.float64), mat2.to(torch.float64)).to(torch.int32)


def int_scaled_matmul(a: torch.Tensor, b: torch.Tensor, scales1: torch.Tensor) -> torch.Tensor:
    """(a @ b) * scales1 with a [M, K] int8, b [K, N] int8, scales1 [M, 1]."""
    M, K = a.shape
    K2, N = b.shape
    assert K == K2, f"inner dimensions differ: {K} vs {K2}"
    assert M == scales1.size(0) or scales1.numel() == 1
    assert scales1.size(1) == 1
    assert scales1.is_contiguous()
    assert a.device == b.device == scales1.device, (
        f"need all tensors on the same device, got {a.device}, {b.device}, {scales1.device}"
    )
    if (
        a.is_cuda
        and not _is_compiling(a)
        and scales1.dtype == torch.bfloat16
        and scales1.numel() == M
        and b.t().is_contiguous()
        and K % 16 == 0
    ):
        ones = torch.ones(N, dtype=torch.bfloat16, device=a.device)
        return torch.ops.torchao.int8_scaled_mm(a.contiguous(), scales1, b.t(), ones, None)
    scales = scales1.expand((M, N))
    if a.device.type == "cpu":  # reference :133-137
        return torch._int_mm(a, b).to(scales.dtype) * scales
    return safe_int_mm(a, b) * scales
