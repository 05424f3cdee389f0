"""int8-dyn LDS-staged GEMM: 128-column tiles (tao_tune_gemm_bn 128) against the 64-column
kernel and the auto policy, per shape; every variant's output checked bit-identical to auto's.
Kernel durations from dispatch events, weights rotated past the MALL.
Usage: python experiments/sweep_i8_bn.py"""

import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from sweep_gemm import kernel_us, make_int8dyn  # noqa: E402
from torchao import _lib  # noqa: E402


def main():
    shapes = [(128, 4096, 4096), (128, 6144, 4096), (128, 14336, 4096), (128, 28672, 4096),
              (256, 14336, 4096), (512, 4096, 4096), (512, 14336, 4096), (128, 4096, 14336)]
    _lib.call("tao_tune_linear_crossover", 1)
    for M, N, K in shapes:
        run, launches = make_int8dyn(M, N, K)
        row = {"M": M, "N": N, "K": K}
        _lib.call("tao_tune_gemm_algo", 0)
        ref = run(0).clone()
        row["auto"] = round(kernel_us(run, launches), 2)
        _lib.call("tao_tune_gemm_algo", 2)
        for bn in (64, 128):
            _lib.call("tao_tune_gemm_bn", bn)
            for bm in (64, 128):
                for sp in (1, 2, 4):
                    for d in ((2, 3) if bn == 128 else (0,)):
                        _lib.call("tao_tune_gemm", bm, 0, sp)
                        _lib.call("tao_tune_gemm_depth", d)
                        key = f"bn{bn}_bm{bm}_s{sp}" + (f"_d{d}" if d else "")
                        if not torch.equal(run(0), ref):
                            row[key] = "MISMATCH"
                            continue
                        row[key] = round(kernel_us(run, launches), 2)
        for name, args in (("tao_tune_gemm", (0, 0, 0)), ("tao_tune_gemm_depth", (0,)),
                           ("tao_tune_gemm_bn", (0,)), ("tao_tune_gemm_algo", (0,))):
            _lib.call(name, *args)
        best = min((v, k) for k, v in row.items() if k.startswith("bn") and v != "MISMATCH")
        row["best"] = best[1]
        print(json.dumps(row), flush=True)
    _lib.call("tao_tune_linear_crossover", 0)


if __name__ == "__main__":
    main()
