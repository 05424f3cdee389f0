"""A/B: the weight-shared tile GEMM (csrc/gemm_tile.hip) against gemm_mfma.hip's kernels.

Kernel durations from dispatch events (tao_profile_*), weights rotated past the 256 MiB MALL
(sweep_gemm.make_*). Per (path, M, N, K): the old kernels' built-in choice (tile mode 1), the tile
kernel at its built-in split and at forced splits, and the outputs' agreement. One JSON line each.

    python experiments/ab_tile.py [--quick]
"""

import json
import sys

import torch

from sweep_gemm import kernel_us, make_int4, make_int8dyn, make_int8wo
from torchao import _lib

LLAMA8B = ((4096, 4096), (6144, 4096), (28672, 4096), (4096, 14336))
QUICK = [("int8dyn", 128, 4096, 4096), ("int4", 128, 4096, 4096), ("int8wo", 128, 4096, 4096),
         ("int4", 128, 28672, 4096)]
FULL = QUICK + [(p, M, N, K) for p in ("int4", "int8dyn", "int8wo") for M in (64, 128, 256, 512)
                for (N, K) in LLAMA8B if (p, M, N, K) not in QUICK]


def main():
    configs = QUICK if "--quick" in sys.argv else FULL
    mk = {"int4": make_int4, "int8wo": make_int8wo, "int8dyn": make_int8dyn}
    for path, M, N, K in configs:
        run, launches = mk[path](M, N, K)
        _lib.call("tao_tune_gemm_tile", 1, 0)
        old_us = kernel_us(run, launches)
        ref = run(0).float()
        rec = {"path": path, "M": M, "N": N, "K": K, "old_us": round(old_us, 2)}
        pts = {}
        for sp in (0, 1, 2, 4, 8, 16):
            _lib.call("tao_tune_gemm_tile", 2, sp)
            pts[sp] = round(kernel_us(run, launches), 2)
            out = run(0).float()
            rel = float((out - ref).norm() / ref.norm().clamp_min(1e-30))
            if rel > 2e-3:
                rec.setdefault("mismatch", {})[sp] = rel
        _lib.call("tao_tune_gemm_tile", 0, 0)
        rec["tile_us"] = pts
        rec["tile_auto_us"] = pts[0]
        rec["speedup"] = round(old_us / pts[0], 2)
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
