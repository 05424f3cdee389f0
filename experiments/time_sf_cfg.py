"""Kernel time of one single-fetch GEMM launch shape (for variant-build A/B runs):

    TORCHAO_MI355X_LIB=... python experiments/time_sf_cfg.py int4 128x28672x4096 128,1,1,3,0,0
prints one JSON line {lib, path, shape, cfg, us} (median of dispatch-packet events, weights
rotated past the MALL as experiments/sweep_sf.py does).
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


def main():
    path, shape, cfg = sys.argv[1], sys.argv[2], sys.argv[3]
    loaders = int(sys.argv[4]) if len(sys.argv) > 4 else 0  # tao_tune_gemm_sf_loaders
    M, N, K = (int(v) for v in shape.split("x"))
    cfg = [int(v) for v in cfg.split(",")]
    gen = torch.Generator(device="cuda").manual_seed(0)
    run, copies = (int8_case if path == "int8" else int4_case)(M, N, K, gen)
    sf(2, *cfg)
    _lib.call("tao_tune_gemm_sf_loaders", loaders)
    us = median(timed(run, copies, 30)) * 1e3
    print(json.dumps({"lib": os.path.basename(os.environ.get("TORCHAO_MI355X_LIB", "shipped")),
                      "path": path, "shape": shape, "cfg": cfg, "loaders": loaders,
                      "us": round(us, 2)}), flush=True)


if __name__ == "__main__":
    main()
