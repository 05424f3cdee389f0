"""Same-process A/B of a two-way single-fetch GEMM knob (1 = off, 2 = on; default the dedicated
LDS-DMA loader waves, KNOB=tao_tune_gemm_sf_xmap for the K-slice -> XCD mapping), per shape and
launch shape, alternated over reps; one JSON line per (case, setting, rep). A cfg of "route" times the built-in route (tao_tune_gemm_sf 0); else
"bn,wm,splits,stages,a_steps,ks[,seam]" under mode 2.

    python experiments/ab_loaders.py [int4:128x4096x4096:route ...]
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

DEFAULT = ["int4:128x4096x4096:route", "int4:128x6144x4096:route", "int4:128x4096x14336:route",
           "int4:128x4096x4096:64,4,4,2,0,0", "int4:128x4096x4096:64,8,4,3,0,0",
           "int4:128x4096x4096:64,2,8,3,0,0,1", "int4:128x4096x14336:64,2,8,3,0,0,1",
           "int8:128x4096x4096:64,4,2,3,0,256", "int8:128x4096x4096:64,4,4,3,0,256,1",
           "int8:128x4096x4096:64,2,4,2,0,128,1", "int8:128x6144x4096:route",
           "int8:128x4096x14336:route"]


def main():
    cases = sys.argv[1:] or DEFAULT
    knob = os.environ.get("KNOB", "tao_tune_gemm_sf_loaders")
    gen = torch.Generator(device="cuda").manual_seed(0)
    for case in cases:
        path, shape, cfg = case.split(":")
        M, N, K = (int(v) for v in shape.split("x"))
        run, copies = (int8_case if path == "int8" else int4_case)(M, N, K, gen)
        if cfg == "route":
            sf(0)
            _lib.call("tao_tune_gemm_sf_seam", -1)
        else:
            c = [int(v) for v in cfg.split(",")]
            sf(2, *c[:6])
            _lib.call("tao_tune_gemm_sf_seam", c[6] if len(c) > 6 else -1)
        ys = {}
        for rep in range(3):
            for ld in (1, 2):
                _lib.call(knob, ld)
                us = median(timed(run, copies, 30)) * 1e3
                if rep == 0:
                    ys[ld] = run(0).clone()
                print(json.dumps({"path": path, "shape": shape, "cfg": cfg, "knob": knob[9:], "set": ld,
                                  "rep": rep, "us": round(us, 2)}), flush=True)
        print(json.dumps({"path": path, "shape": shape, "cfg": cfg,
                          "bit_identical": bool(torch.equal(ys[1], ys[2]))}), flush=True)
        del run
        torch.cuda.empty_cache()
    sf(0)
    _lib.call("tao_tune_gemm_sf_seam", -1)
    _lib.call(knob, 0)


if __name__ == "__main__":
    main()
