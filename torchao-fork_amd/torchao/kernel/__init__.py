from torchao.kernel.intmm import int_scaled_matmul, safe_int_mm

__all__ = ["int_scaled_matmul", "safe_int_mm"]
