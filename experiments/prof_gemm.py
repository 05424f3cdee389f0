"""Run one MFMA skinny-GEMM configuration repeatedly (a target for rocprofv3 counter passes).

python experiments/prof_gemm.py PATH M N K BM KG SPLITS [REPS]
PATH in {int4, int8wo, int8dyn}; BM/KG/SPLITS 0 = auto. Prints the median kernel time.
PROF_SF="mode,bn,wm,splits,stages,a_steps,ks" in the environment sets tao_tune_gemm_sf.
"""

import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "torchao-fork_amd"))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import torch  # noqa: E402

from torchao import _lib  # noqa: E402
from sweep_gemm import kernel_us, make_int4, make_int8dyn, make_int8wo  # noqa: E402


def main():
    path, M, N, K, bm, kg, sp = sys.argv[1], *map(int, sys.argv[2:8])
    reps = int(sys.argv[8]) if len(sys.argv) > 8 else 50
    if len(sys.argv) > 9:  # MFMA GEMM workgroup order (tao_tune_gemm_order)
        _lib.call("tao_tune_gemm_order", int(sys.argv[9]))
    mk = {"int4": make_int4, "int8wo": make_int8wo, "int8dyn": make_int8dyn}[path]
    _lib.call("tao_tune_linear_crossover", 1)
    _lib.call("tao_tune_gemm", bm, kg, sp)
    if os.environ.get("PROF_SF"):  # single-fetch GEMM launch shape: mode,bn,wm,splits,stages,a,ks
        _lib.call("tao_tune_gemm_sf", *[int(v) for v in os.environ["PROF_SF"].split(",")])
    run, launches = mk(M, N, K)
    us = kernel_us(run, launches, reps)
    torch.cuda.synchronize()
    order = sys.argv[9] if len(sys.argv) > 9 else "0"
    print(f"{path} M={M} N={N} K={K} bm={bm} kg={kg} splits={sp} order={order}: {us:.2f} us",
          flush=True)


if __name__ == "__main__":
    main()
