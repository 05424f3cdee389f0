from torchao.kernel.intmm import int_scaled_matmul, safe_int_mm
from torchao.kernel.tuning import reset as reset_tuning
from torchao.kernel.tuning import tuning

__all__ = ["int_scaled_matmul", "safe_int_mm", "tuning", "reset_tuning"]
