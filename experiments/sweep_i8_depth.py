"""int8-dyn LDS-staged GEMM: register-ring depth (tao_tune_gemm_depth) x M tile x K splits per
shape, against the auto policy. Kernel durations from dispatch events, weights rotated past the
MALL. Usage: python experiments/sweep_i8_depth.py"""

import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from sweep_gemm import kernel_us, make_int8dyn  # noqa: E402
from torchao import _lib  # noqa: E402


def main():
    shapes = [(128, 4096, 4096), (128, 6144, 4096), (128, 14336, 4096), (128, 4096, 14336),
              (256, 4096, 4096), (512, 4096, 4096)]
    _lib.call("tao_tune_linear_crossover", 1)
    for M, N, K in shapes:
        run, launches = make_int8dyn(M, N, K)
        row = {"M": M, "N": N, "K": K}
        _lib.call("tao_tune_gemm_algo", 0)
        row["auto"] = round(kernel_us(run, launches), 2)
        _lib.call("tao_tune_gemm_algo", 2)
        for bm in (64, 128):
            for sp in (1, 2, 4):
                for d in ((2, 3, 4, 6, 8) if bm == 64 else (2, 3, 4, 6)):
                    _lib.call("tao_tune_gemm", bm, 0, sp)
                    _lib.call("tao_tune_gemm_depth", d)
                    row[f"bm{bm}_s{sp}_d{d}"] = round(kernel_us(run, launches), 2)
        _lib.call("tao_tune_gemm", 0, 0, 0)
        _lib.call("tao_tune_gemm_depth", 0)
        _lib.call("tao_tune_gemm_algo", 0)
        best = min((v, k) for k, v in row.items() if k.startswith("bm"))
        row["best"] = best[1]
        print(json.dumps(row), flush=True)
    _lib.call("tao_tune_linear_crossover", 0)


if __name__ == "__main__":
    main()
