"""int8 matmul entry points (reference torchao/kernel/intmm.py:30-143).

``int_scaled_matmul(a, b, scales1)`` = ``(a @ b) * scales1`` with int32 accumulation. On the GPU
with bf16 row scales and a ``b`` that is the transpose of a contiguous [N, K] weight (the shape
every int8 linear produces) it runs the gfx950 int8-MFMA kernel with the scale fused in its
epilogue; other inputs use ``torch._int_mm`` (hipBLASLt on ROCm), as the reference does.
The Triton autotuner path of the reference (``TORCHAO_AUTOTUNER_ENABLE``) does not exist here.
"""

import torch

__all__ = ["safe_int_mm", "int_scaled_matmul"]


def safe_int_mm(input: torch.Tensor, mat2: torch.Tensor) -> torch.Tensor:
    """int8 [M, K] @ int8 [K, N] -> int32 [M, N]."""
    assert input.dtype == torch.int8 and mat2.dtype == torch.int8
    if input.device.type == "cpu" or input.shape[0] <= 16:
        # torch._int_mm's ROCm/CPU kernels reject tiny M; widen and multiply exactly in int32
        return torch.mm(input.to(torch.int32), mat2.to(torch.int32)) if input.device.type != "cpu" \
            else torch._int_mm(input, mat2)
    return torch._int_mm(input, mat2)


def int_scaled_matmul(a: torch.Tensor, b: torch.Tensor, scales1: torch.Tensor) -> torch.Tensor:
    """(a @ b) * scales1 with a [M, K] int8, b [K, N] int8, scales1 [M, 1]."""
    M, K = a.shape
    K2, N = b.shape
    assert K == K2
    assert M == scales1.size(0) or scales1.numel() == 1
    assert scales1.size(1) == 1
    assert scales1.is_contiguous()
    if (
        a.is_cuda
        and scales1.dtype == torch.bfloat16
        and scales1.numel() == M
        and b.t().is_contiguous()
        and K % 16 == 0
    ):
        ones = torch.ones(N, dtype=torch.bfloat16, device=a.device)
        return torch.ops.torchao.int8_scaled_mm(a.contiguous(), scales1, b.t(), ones, None)
    scales = scales1.expand((M, N))
    if a.device.type == "cpu":
        return torch._int_mm(a, b).to(scales.dtype) * scales
    return safe_int_mm(a, b) * scales
