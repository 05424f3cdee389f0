"""Time the stream prefill GEMM (tao_tune_gemm_stream 2) at the M = 128 Llama-3-8B shapes.

One JSON line per (path, N, K): kernel µs from dispatch events, weights rotated past the MALL.
    python experiments/prof_stream.py [--variant V] [--mode 2]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from sweep_gemm import kernel_us, make_int4, make_int8dyn  # noqa: E402
from torchao import _lib  # noqa: E402

CFGS = [("int8dyn", 128, 4096, 4096), ("int4", 128, 4096, 4096), ("int8dyn", 128, 28672, 4096),
        ("int4", 128, 28672, 4096)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variant", type=int, default=0)
    ap.add_argument("--mode", type=int, default=2)
    a = ap.parse_args()
    mk = {"int4": make_int4, "int8dyn": make_int8dyn}
    for path, M, N, K in CFGS:
        run, launches = mk[path](M, N, K)
        _lib.call("tao_tune_gemm_stream", a.mode)
        us = kernel_us(run, launches, reps=24)
        _lib.call("tao_tune_gemm_stream", 0)
        print(json.dumps({"variant": a.variant, "mode": a.mode, "path": path, "M": M, "N": N,
                          "K": K, "us": round(us, 2)}), flush=True)


if __name__ == "__main__":
    main()
