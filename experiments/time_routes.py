"""Kernel time of the routed prefill GEMMs (tao_tune_gemm_sf mode 0: the built-in routes) at M=128
for the Llama-3-8B and -70B linear shapes, int8 dyn and int4 g32 (dispatch-packet events, median
of 30, weights rotated past the MALL as experiments/sweep_sf.py does):
    [TORCHAO_MI355X_LIB=...] python experiments/time_routes.py [--big] >> out.jsonl
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "torchao-fork_amd"))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import torch  # noqa: E402

from sweep_sf import int4_case, int8_case, median, sf, timed  # noqa: E402
from torchao import _lib  # noqa: E402

SHAPES_8B = [(4096, 4096), (6144, 4096), (28672, 4096), (4096, 14336)]
SHAPES_70B = [(10240, 8192), (8192, 8192), (57344, 8192), (8192, 28672)]


def main():
    lib = os.path.basename(os.environ.get("TORCHAO_MI355X_LIB", "shipped"))
    shapes = SHAPES_8B + (SHAPES_70B if "--big" in sys.argv else [])
    gen = torch.Generator(device="cuda").manual_seed(0)
    for path in ("int8", "int4"):
        for N, K in shapes:
            run, copies = (int8_case if path == "int8" else int4_case)(128, N, K, gen)
            _lib.call("tao_tune_reset")
            sf(0)
            us = median(timed(run, copies, 30)) * 1e3
            print(json.dumps({"lib": lib, "path": path, "M": 128, "N": N, "K": K, "us": round(us, 2)}),
                  flush=True)
            del run
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
