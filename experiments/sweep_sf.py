"""Sweep of the single-fetch prefill GEMM (csrc/gemm_sf.hip) against the routed incumbent.

Per (path, M, N, K) and launch shape (bn, wm, splits, stages, a_steps, ks): kernel us from the
dispatch packets' own events (tao_profile_*, what rocprofv3 reports), median over reps, weights
rotated over copies past the 256 MiB MALL (as bench.py prefill_mfma times them). Outputs are
checked against the incumbent kernel (int8 dyn bit-exact; int4 within 2e-3 rel. L2).

    python experiments/sweep_sf.py [--quick] [--out gpurun_out/sf_sweep.jsonl]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "torchao-fork_amd"))
import torch  # noqa: E402

import torchao  # noqa: E402,F401
from torchao import _lib  # noqa: E402

DEV = "cuda"


def sf(mode, bn=0, wm=0, splits=0, stages=0, a=0, ks=0):
    _lib.call("tao_tune_gemm_sf", mode, bn, wm, splits, stages, a, ks)


def timed(fn, copies, reps):
    for c in range(copies):
        fn(c)
    torch.cuda.synchronize()
    with _lib.KernelTimer(reps * 4) as kt:
        for i in range(reps):
            fn(i % copies)
    torch.cuda.synchronize()
    d = kt.durations_ms
    return d


def int8_case(M, N, K, gen):
    copies = max(2, int(320e6 // (N * K)))
    ws = [torch.randint(-127, 128, (N, K), dtype=torch.int8, device=DEV, generator=gen)
          for _ in range(copies)]
    wsc = (torch.rand(N, device=DEV, generator=gen) * 0.01 + 1e-3).to(torch.bfloat16)
    x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16, generator=gen)
    xq, xs = torch.ops.torchao.int8_quantize_per_token(x)

    def run(c):
        return torch.ops.torchao.int8_scaled_mm(xq, xs, ws[c], wsc, None)
    return run, copies


def int4_case(M, N, K, gen, g=32):
    copies = max(2, int(320e6 // (N * K // 2)))
    w4 = []
    for _ in range(copies):
        q = torch.randint(0, 16, (N, K), dtype=torch.int32, device=DEV, generator=gen)
        sz = (torch.rand(N, K // g, 2, device=DEV, generator=gen) * 0.02).to(torch.bfloat16)
        w4.append((torch.ops.torchao.int4_pack(q), sz))
        del q
    x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16, generator=gen)

    def run(c):
        return torch.ops.torchao.int4_weight_only_linear(x, w4[c][0], w4[c][1], g, None)
    return run, copies


def median(v):
    v = sorted(v)
    return v[len(v) // 2] if v else float("nan")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--quick", action="store_true")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "sf_sweep.jsonl"))
    ap.add_argument("--paths", default="int8,int4")
    ap.add_argument("--shapes", default="")
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--seams", default="1,0", help="split-K seams to time (1 spread, 0 fixed reducer)")
    ap.add_argument("--cfgs", default="", help="launch shapes to time, ';'-separated (default: the built-in list)")
    args = ap.parse_args()
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    out = open(args.out, "a")
    gen = torch.Generator(device=DEV).manual_seed(0)
    shapes = [(128, 4096, 4096)]
    if not args.quick:
        shapes += [(128, 6144, 4096), (128, 28672, 4096), (128, 4096, 14336), (64, 4096, 4096)]
    if args.shapes:
        shapes = [tuple(int(v) for v in s.split("x")) for s in args.shapes.split(",")]
    cfgs = {
        "int8": [(32, 8, 2, 3, 0, 256), (32, 4, 2, 3, 0, 256), (32, 8, 2, 2, 0, 256),
                 (32, 8, 2, 4, 0, 256), (32, 8, 4, 3, 0, 256), (64, 4, 4, 3, 0, 128),
                 (64, 4, 4, 4, 0, 128), (64, 8, 4, 3, 0, 128), (64, 2, 4, 3, 0, 128),
                 (64, 4, 2, 3, 0, 256), (64, 4, 4, 2, 0, 256), (128, 4, 8, 3, 0, 128),
                 (128, 2, 8, 3, 0, 128), (128, 4, 8, 2, 0, 256), (64, 4, 1, 3, 0, 128),
                 (32, 8, 1, 3, 0, 256), (32, 8, 2, 3, 9, 256), (32, 8, 2, 3, 7, 256),
                 (256, 2, 2, 2, 0, 128), (256, 4, 2, 3, 0, 128), (256, 2, 1, 3, 0, 128),
                 (256, 4, 4, 2, 0, 128), (256, 2, 4, 3, 0, 128)],
        "int4": [(64, 2, 4, 3, 0), (64, 4, 4, 3, 0), (64, 8, 4, 3, 0), (64, 2, 4, 2, 0),
                 (64, 2, 4, 4, 0), (128, 2, 8, 2, 0), (128, 2, 8, 3, 0), (128, 4, 8, 3, 0),
                 (128, 8, 8, 3, 0), (64, 2, 2, 3, 0), (128, 2, 4, 3, 0), (64, 2, 8, 3, 0),
                 (64, 2, 4, 3, 9), (128, 4, 8, 3, 5), (128, 1, 8, 2, 0), (128, 1, 4, 3, 0),
                 (128, 1, 2, 3, 0), (128, 1, 1, 3, 0), (64, 1, 4, 2, 0), (64, 1, 2, 3, 0),
                 (64, 1, 8, 2, 0), (128, 1, 8, 3, 0),
                 (256, 2, 2, 2, 0), (256, 2, 2, 3, 0), (256, 2, 1, 3, 0), (256, 4, 2, 2, 0),
                 (256, 2, 4, 2, 0), (256, 4, 4, 3, 0), (256, 2, 8, 2, 0),
                 (128, 1, 1, 3, 0, 2), (128, 1, 1, 2, 0, 2), (128, 1, 2, 3, 0, 2),
                 (128, 1, 4, 2, 0, 2), (128, 1, 4, 3, 0, 2), (128, 1, 8, 2, 0, 2)],
    }
    if args.cfgs:
        own = [tuple(int(v) for v in c.split(",")) for c in args.cfgs.split(";")]
        cfgs = {p: own for p in cfgs}
    lib = os.path.basename(os.environ.get("TORCHAO_MI355X_LIB", "shipped"))
    for path in args.paths.split(","):
        for (M, N, K) in shapes:
            run, copies = (int8_case if path == "int8" else int4_case)(M, N, K, gen)
            base = None
            for cs in ((32,) if args.cfgs else (1, 32)):  # split-K tickets packed / one 128-B line per tile
                _lib.call("tao_tune_reset")
                sf(1)
                _lib.call("tao_tune_cnt_stride", cs)
                if base is None:
                    ref = run(0).clone()
                t = median(timed(run, copies, args.reps))
                base = t if base is None else base
                rec = {"lib": lib, "path": path, "M": M, "N": N, "K": K, "cfg": "incumbent", "cs": cs,
                       "us": round(t * 1e3, 2)}
                print(json.dumps(rec), flush=True)
                out.write(json.dumps(rec) + "\n")
            seams = [int(v) for v in args.seams.split(",")]
            todo = [(c, sm) for c in cfgs[path] for sm in seams if sm == 0 or c[2] in (2, 4, 8)]
            for cfg, seam in todo:
                _lib.call("tao_tune_reset")
                try:
                    sf(2, *cfg)
                    _lib.call("tao_tune_gemm_sf_seam", seam)
                    y = run(0)
                    torch.cuda.synchronize()
                    if path == "int8":
                        ok = bool(torch.equal(y, ref))
                    else:
                        ok = float((y.float() - ref.float()).norm() / ref.float().norm()) < 2e-3
                    us = median(timed(run, copies, args.reps)) * 1e3
                    rec = {"lib": lib, "path": path, "M": M, "N": N, "K": K, "cfg": list(cfg), "seam": seam,
                           "us": round(us, 2), "speedup": round(base * 1e3 / us, 3), "ok": ok}
                except RuntimeError as e:
                    rec = {"path": path, "M": M, "N": N, "K": K, "cfg": list(cfg), "error": str(e)[:120]}
                print(json.dumps(rec), flush=True)
                out.write(json.dumps(rec) + "\n")
            st = torch.zeros(1, dtype=torch.int32)
            _lib.call("tao_gemm_sf_status", st.data_ptr())
            if int(st.item()):
                print(json.dumps({"sf_status": int(st.item())}), flush=True)
            del run
            torch.cuda.empty_cache()
    _lib.call("tao_tune_reset")


if __name__ == "__main__":
    t0 = time.time()
    main()
    print(json.dumps({"elapsed_s": round(time.time() - t0, 1)}))
