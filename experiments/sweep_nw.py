"""Columns per wave (tao_tune_gemm_nw) x launch shape sweep of the MFMA skinny GEMM.

For every configuration and every (bm, kg, splits), the 16-column (nw 1) and the 32-column
(nw 2) kernel are timed (dispatch events, weights rotated past the MALL) and their outputs
compared: the per-element accumulation order does not depend on nw, so they must be equal.
One JSON line per configuration: auto time, best per nw, and every point. For int4 the
32x32x16 kernel (tao_tune_int4_mfma32) is swept too, recorded with nw = 32.

    python experiments/sweep_nw.py [--quick] [--wide | --wide70 | --int4]
    (--wide: 3 paths x 6 M x the Llama-3-8B linears; --wide70: the 70B linears and heads, plus
    int8-dyn at the 8B shapes with the product path's own kernel choice as "auto")
"""

import itertools
import json
import sys

import torch

from sweep_gemm import kernel_us, make_int4, make_int8dyn, make_int8wo
from torchao import _lib

CONFIGS = [
    ("int4", 128, 4096, 4096), ("int4", 128, 6144, 4096), ("int4", 128, 28672, 4096),
    ("int4", 128, 4096, 14336), ("int4", 64, 4096, 4096), ("int4", 256, 4096, 4096),
    ("int4", 512, 4096, 4096), ("int4", 32, 4096, 4096), ("int4", 128, 128256, 4096),
    ("int8dyn", 128, 4096, 4096), ("int8dyn", 128, 28672, 4096), ("int8wo", 128, 4096, 4096),
    ("int8wo", 128, 28672, 4096),
]
LLAMA8B = ((4096, 4096), (6144, 4096), (28672, 4096), (4096, 14336))
LLAMA70B = ((10240, 8192), (8192, 8192), (57344, 8192), (8192, 28672), (128256, 4096),
            (128256, 8192))
MS = (16, 32, 64, 128, 256, 512)
WIDE = [(p, M, N, K) for p in ("int4", "int8wo", "int8dyn") for M in MS for (N, K) in LLAMA8B]
INT4 = [("int4", M, N, K) for M in MS for (N, K) in LLAMA8B + LLAMA70B]
WIDE70 = ([(p, M, N, K) for p in ("int4", "int8wo", "int8dyn") for M in MS for (N, K) in LLAMA70B]
          + [("int8dyn", M, N, K) for M in MS for (N, K) in LLAMA8B])


def main():
    quick = "--quick" in sys.argv
    configs = (WIDE if "--wide" in sys.argv else WIDE70 if "--wide70" in sys.argv
               else INT4 if "--int4" in sys.argv else CONFIGS)
    mk = {"int4": make_int4, "int8wo": make_int8wo, "int8dyn": make_int8dyn}
    _lib.call("tao_tune_linear_crossover", 1)
    for path, M, N, K in configs[:4] if quick else configs:
        run, launches = mk[path](M, N, K)
        _lib.call("tao_tune_gemm", 0, 0, 0)
        _lib.call("tao_tune_gemm_nw", 0)
        _lib.call("tao_tune_gemm_algo", 0)  # the product path (int8-dyn: either kernel)
        rec = {"path": path, "M": M, "N": N, "K": K, "auto_us": round(kernel_us(run, launches), 2)}
        _lib.call("tao_tune_gemm_algo", 1)  # int8-dyn: the template kernel (the one nw applies to)
        pts = []
        best = {1: (1e9, None), 2: (1e9, None)}
        mismatches = []
        for bm, kg, sp in itertools.product((16, 32, 64, 128), (1, 2), (1, 2, 4, 8)):
            if bm > M * 2 or (bm == 64 and kg == 2 and path == "int4" and sp > 2):
                continue
            if bm == 128 and (path == "int4" or kg > 1):
                continue
            _lib.call("tao_tune_gemm", bm, kg, sp)
            outs = {}
            for nw in ((1,) if bm == 128 else (1, 2)):
                _lib.call("tao_tune_gemm_nw", nw)
                us = kernel_us(run, launches)
                outs[nw] = run(0).clone()
                pts.append([bm, kg, sp, nw, round(us, 2)])
                if us < best[nw][0]:
                    best[nw] = (round(us, 2), [bm, kg, sp])
            if 2 in outs and not torch.equal(outs[1], outs[2]):
                mismatches.append([bm, kg, sp])
        if path == "int4":  # the 32x32x16 kernel, recorded as nw 32
            _lib.call("tao_tune_gemm_nw", 0)
            _lib.call("tao_tune_int4_mfma32", 1)
            for bm, sp in itertools.product((32, 64), (1, 2, 4, 8)):
                _lib.call("tao_tune_gemm", bm, 0, sp)
                pts.append([bm, 1, sp, 32, round(kernel_us(run, launches), 2)])
            _lib.call("tao_tune_int4_mfma32", 0)
        _lib.call("tao_tune_gemm", 0, 0, 0)
        _lib.call("tao_tune_gemm_nw", 0)
        _lib.call("tao_tune_gemm_algo", 0)
        rec["best_nw1"] = best[1]
        rec["best_nw2"] = best[2]
        rec["nw_mismatch"] = mismatches
        rec["points"] = pts
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
