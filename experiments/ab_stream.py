"""A/B: the stream prefill GEMM (csrc/gemm_stream.hip) against the built-in routing without it.

Kernel durations from dispatch events (tao_profile_*), weights rotated past the 256 MiB MALL
(sweep_gemm.make_*). Per (path, M, N, K): the previous routing (stream mode 1), the stream kernel
(mode 2), their outputs' agreement. One JSON line each.

    python experiments/ab_stream.py [--quick]
"""

import json
import sys

from sweep_gemm import kernel_us, make_int4, make_int8dyn
from torchao import _lib

LLAMA8B = ((4096, 4096), (6144, 4096), (28672, 4096), (4096, 14336))
QUICK = [("int8dyn", 128, 4096, 4096), ("int4", 128, 4096, 4096), ("int4", 128, 28672, 4096),
         ("int8dyn", 128, 28672, 4096)]
FULL = QUICK + [(p, M, N, K) for p in ("int4", "int8dyn") for M in (33, 64, 96, 128, 192, 256, 512)
                for (N, K) in LLAMA8B if (p, M, N, K) not in QUICK]


def main():
    configs = QUICK if "--quick" in sys.argv else FULL
    mk = {"int4": make_int4, "int8dyn": make_int8dyn}
    for path, M, N, K in configs:
        run, launches = mk[path](M, N, K)
        _lib.call("tao_tune_gemm_stream", 1)
        old_us = kernel_us(run, launches)
        ref = run(0).float()
        row = {"path": path, "M": M, "N": N, "K": K, "old_us": round(old_us, 2)}
        for mode, key in ((2, "stream"), (4, "stream_rot_m"), (5, "stream_rot_mn")):
            _lib.call("tao_tune_gemm_stream", mode)
            us = kernel_us(run, launches)
            out = run(0).float()
            row[f"{key}_us"] = round(us, 2)
            row[f"{key}_rel_vs_old"] = float((out - ref).norm() / ref.norm().clamp_min(1e-30))
        _lib.call("tao_tune_gemm_stream", 0)
        row["speedup"] = round(old_us / min(row["stream_us"], row["stream_rot_m_us"],
                                            row["stream_rot_mn_us"]), 2)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
