"""int8-dyn GEMM: the LDS-staged kernel (tao_tune_gemm_algo 2) against the per-wave-column MFMA
kernel (algo 1) per shape, every (M tile, K splits) of the LDS kernel; kernel durations from
dispatch events, weights rotated past the MALL. Usage: python experiments/sweep_i8_lds.py"""

import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from sweep_gemm import kernel_us, make_int8dyn  # noqa: E402
from torchao import _lib  # noqa: E402


def main():
    shapes = [(128, 4096, 4096), (128, 14336, 4096), (128, 4096, 14336), (64, 4096, 4096),
              (256, 4096, 4096), (512, 4096, 4096), (128, 6144, 4096), (128, 28672, 4096)]
    _lib.call("tao_tune_linear_crossover", 1)
    for M, N, K in shapes:
        run, launches = make_int8dyn(M, N, K)
        row = {"M": M, "N": N, "K": K}
        for algo in (0, 1, 2):  # 0: the shipped auto policy
            _lib.call("tao_tune_gemm_algo", algo)
            _lib.call("tao_tune_gemm", 0, 0, 0)
            row[f"auto_algo{algo}"] = round(kernel_us(run, launches), 2)
        _lib.call("tao_tune_gemm_algo", 2)
        for bm in (64, 128):
            for sp in (1, 2, 4, 8, 16):
                _lib.call("tao_tune_gemm", bm, 0, sp)
                row[f"lds_bm{bm}_s{sp}"] = round(kernel_us(run, launches), 2)
        _lib.call("tao_tune_gemm", 0, 0, 0)
        _lib.call("tao_tune_gemm_algo", 0)
        print(json.dumps(row), flush=True)
    _lib.call("tao_tune_linear_crossover", 0)


if __name__ == "__main__":
    main()
