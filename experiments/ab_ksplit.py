"""A/B: the k-split prefill GEMM (csrc/gemm_ksplit.hip) against the built-in routing without it.

Kernel durations from dispatch events (tao_profile_*), weights rotated past the 256 MiB MALL
(sweep_gemm.make_*). Per (path, M, N, K): the previous routing (k-split mode 1), the k-split
kernel at each launch shape (mode 2, shape 1..3), their outputs' agreement. One JSON line each.

    python experiments/ab_ksplit.py [--quick]
"""

import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from sweep_gemm import kernel_us, make_int4, make_int8dyn  # noqa: E402
from torchao import _lib  # noqa: E402

LLAMA8B = ((4096, 4096), (6144, 4096), (28672, 4096), (4096, 14336))
QUICK = [("int8dyn", 128, 4096, 4096), ("int4", 128, 4096, 4096), ("int4", 128, 28672, 4096),
         ("int8dyn", 128, 28672, 4096), ("int4", 128, 4096, 14336), ("int8dyn", 128, 6144, 4096)]
FULL = QUICK + [(p, M, N, K) for p in ("int4", "int8dyn") for M in (32, 64, 96, 128, 192, 256, 512)
                for (N, K) in LLAMA8B if (p, M, N, K) not in QUICK]


SHAPES = (1, 2, 3, 4)


def main():
    global SHAPES
    if "--rot" in sys.argv:
        SHAPES = (1, 17, 2, 18, 3, 19)
    configs = QUICK if "--quick" in sys.argv else FULL
    mk = {"int4": make_int4, "int8dyn": make_int8dyn}
    for path, M, N, K in configs:
        run, launches = mk[path](M, N, K)
        _lib.call("tao_tune_gemm_ksplit", 1, 0)
        old_us = kernel_us(run, launches)
        ref = run(0).float()
        row = {"path": path, "M": M, "N": N, "K": K, "old_us": round(old_us, 2)}
        best = None
        for shape in SHAPES:
            _lib.call("tao_tune_gemm_ksplit", 2, shape)
            us = kernel_us(run, launches)
            out = run(0).float()
            rel = float((out - ref).norm() / ref.norm().clamp_min(1e-30))
            row[f"ksplit{shape}_us"] = round(us, 2)
            row[f"ksplit{shape}_rel"] = rel
            if best is None or us < best[0]:
                best = (us, shape)
        _lib.call("tao_tune_gemm_ksplit", 0, 0)
        row["best_shape"] = best[1]
        row["speedup"] = round(old_us / best[0], 2)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
