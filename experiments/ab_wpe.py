"""MFMA GEMM occupancy A/B: run under the in-tree library and under a TAO_GEMM_WPE build
(TORCHAO_MI355X_LIB); prints kernel us for forced (bm, kg, splits) shapes.

    python experiments/ab_wpe.py TAG
"""
import json
import sys

from sweep_gemm import kernel_us, make_int4, make_int8dyn
from torchao import _lib

tag = sys.argv[1] if len(sys.argv) > 1 else "lib"
_lib.call("tao_tune_linear_crossover", 1)
_lib.call("tao_tune_gemm_algo", 1)
for path, M, N, K in [("int4", 128, 4096, 4096), ("int4", 64, 4096, 4096), ("int4", 128, 6144, 4096),
                      ("int4", 128, 28672, 4096), ("int4", 32, 4096, 4096),
                      ("int8dyn", 128, 4096, 4096)]:
    run, launches = (make_int4 if path == "int4" else make_int8dyn)(M, N, K)
    rec = {"tag": tag, "path": path, "M": M, "N": N, "K": K}
    for bm, kg, sp in [(32, 1, 1), (32, 1, 2), (32, 1, 4), (32, 1, 8), (16, 1, 4), (32, 2, 1),
                       (64, 1, 4)]:
        _lib.call("tao_tune_gemm", bm, kg, sp)
        rec[f"{bm}_{kg}_{sp}"] = round(kernel_us(run, launches, reps=30), 2)
    _lib.call("tao_tune_gemm", 0, 0, 0)
    print(json.dumps(rec), flush=True)
