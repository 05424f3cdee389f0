"""int4 GEMM: gemm_mfma_kernel (16x16x32, built-in shape incl. the measured table) vs
gemm32_int4_kernel (32x32x16) at its auto shape and forced (bm, splits); kernel us.

    python experiments/ab_mfma32.py
"""
import json

from sweep_gemm import kernel_us, make_int4
from torchao import _lib

CONFIGS = [(128, 4096, 4096), (128, 6144, 4096), (128, 28672, 4096), (128, 4096, 14336),
           (64, 4096, 4096), (32, 4096, 4096), (256, 4096, 4096), (512, 4096, 4096),
           (512, 28672, 4096), (16, 4096, 4096)]


def main():
    _lib.call("tao_tune_linear_crossover", 1)
    for M, N, K in CONFIGS:
        run, launches = make_int4(M, N, K)
        rec = {"M": M, "N": N, "K": K}
        _lib.call("tao_tune_int4_mfma32", 0)
        rec["mfma16_us"] = round(kernel_us(run, launches, reps=30), 2)
        _lib.call("tao_tune_int4_mfma32", 1)
        rec["mfma32_auto_us"] = round(kernel_us(run, launches, reps=30), 2)
        pts = []
        for bm in (32, 64, 128):
            for sp in (1, 2, 4, 8):
                _lib.call("tao_tune_gemm", bm, 0, sp)
                pts.append([bm, sp, round(kernel_us(run, launches, reps=30), 2)])
        _lib.call("tao_tune_gemm", 0, 0, 0)
        _lib.call("tao_tune_int4_mfma32", 0)
        rec["mfma16_again_us"] = round(kernel_us(run, launches, reps=30), 2)
        rec["mfma32_best"] = min(pts, key=lambda p: p[2])
        rec["mfma32_points"] = pts
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
