"""Per-step timeline of the 32x32x16 int4 prefill GEMM (gemm_sf32.hip built with
TAO_SF32_STEPSTAMPS=1: experiments/variant.sh steps=gemm_sf32:-DTAO_SF32_STEPSTAMPS=1): for every
wave of workgroups 0..7 of the last of several launches, s_memtime at each k step's top, after its
own DMAs landed (vmcnt), after the step barrier, after the step's MFMAs were issued. Prints one
JSON line per shape: median cycles per step in each phase, the in-kernel clock, span.

    TORCHAO_MI355X_LIB=experiments/build/libvar_steps.so python experiments/sf32_steps.py
"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "torchao-fork_amd"))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from sweep_sf import int4_case, sf  # noqa: E402
from torchao import _lib  # noqa: E402

lib = _lib.lib()
lib.tao_debug_sf32_steps.argtypes = [ctypes.c_void_p]
NWG, NWV, NST = 8, 8, 64


def main():
    # (shape, launch shape, tao_tune_gemm_sf_loaders): with loaders (2) waves 0-3 compute and
    # 4-7 load; their phases are reported separately
    cases = [("128x28672x4096", (128, 1, 1, 3, 0, 0), 1), ("128x28672x4096", (128, 1, 1, 3, 0, 0), 2),
             ("128x28672x4096", (128, 1, 1, 3, 0, 2), 1), ("128x57344x8192", (256, 1, 1, 3, 0, 0), 1)]
    gen = torch.Generator(device="cuda").manual_seed(0)
    buf = np.zeros(NWG * NWV * NST * 4 + NWG * NWV * 4, dtype=np.uint64)
    for shape, cfg, ld in cases:
        M, N, K = (int(v) for v in shape.split("x"))
        run, copies = int4_case(M, N, K, gen)
        sf(2, *cfg)
        lib.tao_tune_gemm_sf_loaders(ld)
        for c in range(copies):
            run(c)
        torch.cuda.synchronize()
        lib.tao_debug_sf32_steps(buf.ctypes.data)  # clear
        run(0)
        torch.cuda.synchronize()
        assert lib.tao_debug_sf32_steps(buf.ctypes.data) == 0
        ts = buf[:NWG * NWV * NST * 4].reshape(NWG, NWV, NST, 4).astype(np.int64)
        te = buf[NWG * NWV * NST * 4:].reshape(NWG, NWV, 4).astype(np.int64)
        nsteps = K // 128
        waves = 4 * (2 if cfg[5] == 2 else 1) * (2 if cfg[0] == 256 else 1)
        t = ts[:, :waves, 1:min(nsteps, NST) - 1, :]  # steady steps
        wait = t[..., 1] - t[..., 0]
        bar = t[..., 2] - t[..., 1]
        comp = t[..., 3] - t[..., 2]
        step = np.diff(ts[:, :waves, :min(nsteps, NST), 0], axis=-1)
        span_cyc = te[:, :waves, 2] - te[:, :waves, 0]
        span_rt = (te[:, :waves, 3] - te[:, :waves, 1]) * 10.0  # ns (100 MHz)
        clk = float(np.median(span_cyc / np.maximum(span_rt, 1)))  # GHz
        if ld == 2:
            lt = ts[:, waves:2 * waves, 1:min(nsteps, NST) - 1, :]
            loader = {"loader_wait_dma_cyc": float(np.median(lt[..., 1] - lt[..., 0])),
                      "loader_barrier_cyc": float(np.median(lt[..., 2] - lt[..., 1])),
                      "loader_issue_cyc": float(np.median(lt[..., 3] - lt[..., 2]))}
        else:
            loader = {}
        rec = {"shape": shape, "cfg": list(cfg), "loaders": ld, "waves": waves, "steps": nsteps,
               "clock_GHz": round(clk, 3),
               "cyc_per_step_median": float(np.median(step)),
               "wait_dma_cyc": float(np.median(wait)), "barrier_cyc": float(np.median(bar)),
               "compute_issue_cyc": float(np.median(comp)),
               "wait_dma_p90": float(np.percentile(wait, 90)),
               "barrier_p90": float(np.percentile(bar, 90)),
               "span_us_median": round(float(np.median(span_rt)) / 1e3, 2),
               "first_step_wait_cyc": float(np.median(ts[:, :waves, 0, 1] - ts[:, :waves, 0, 0])),
               **loader}
        print(json.dumps(rec), flush=True)
        sf(0)
        lib.tao_tune_gemm_sf_loaders(0)
        del run


if __name__ == "__main__":
    main()
