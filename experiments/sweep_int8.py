"""Sweep the M = 1 launch shape of the int8 decode GEMVs (tao_tune_int8_gemv) per weight shape:
int8 weight-only (bf16 x) and the fused int8 x int8 one-token linear (int8_dyn_linear).
Weights rotated past the Infinity Cache, one dispatch-event timing per launch (KernelTimer),
median; every config's output is checked against the default (int8 dyn: bit-exact).
--graph: time by the wall time per launch of back-to-back launches replayed from one HIP graph
(sweep_gemv.graph_us), as bench.py's int8wo_m1 block does.
python experiments/sweep_int8.py [--graph] [NxK ...]"""

import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "torchao-fork_amd"))
import torch  # noqa: E402

import torchao  # noqa: E402,F401
from torchao import _lib  # noqa: E402

SHAPES = [(6144, 4096), (4096, 4096), (28672, 4096), (4096, 14336), (128256, 4096)]


def main():
    args = [a for a in sys.argv[1:] if a != "--graph"]
    use_graph = "--graph" in sys.argv[1:]
    if use_graph:
        sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
        from sweep_gemv import graph_us
    shapes = SHAPES if not args else [tuple(map(int, a.split("x"))) for a in args]
    for N, K in shapes:
        S = (K // 16 + 63) // 64
        copies = max(3, min(48, int(400e6 // (N * K))))
        ws = [torch.randint(-127, 128, (N, K), dtype=torch.int8, device="cuda") for _ in range(copies)]
        sc = (torch.rand(N, device="cuda") * 0.01 + 1e-3).to(torch.bfloat16)
        x = torch.randn(1, K, device="cuda", dtype=torch.bfloat16)
        reps = max(copies, 40)
        paths = {
            "int8wo": lambda w: torch.ops.torchao.int8_weight_only_linear(x, w, sc, None),
            "int8dyn_fused": lambda w: torch.ops.torchao.int8_dyn_linear(x, w, sc, None),
        }
        for name, fn in paths.items():
            _lib.call("tao_tune_int8_gemv", 0, 0, 0)
            ref = fn(ws[0]).float()
            res = []
            cfgs = [(0, 0, 0)] + [(rpw, wk, g) for rpw in (2, 4, 8)
                                  for wk in sorted({w for w in (1, 2, 4, 8) if w <= S} | {min(S, 8)})
                                  for g in (1, 2, 4, 8) if wk * g <= 8]
            for rpw, wk, g in cfgs:
                if True:
                    if True:
                        _lib.call("tao_tune_int8_gemv", rpw, wk, g)
                        out = fn(ws[0]).float()
                        err = float((out - ref).norm() / ref.norm().clamp_min(1e-30))
                        for c in range(copies):
                            fn(ws[c])
                        torch.cuda.synchronize()
                        if use_graph:
                            us = graph_us(lambda: [fn(ws[i % copies]) for i in range(reps)], reps)
                        else:
                            with _lib.KernelTimer(reps) as kt:
                                for i in range(reps):
                                    fn(ws[i % copies])
                            us = statistics.median(kt.durations_ms[2:]) * 1e3
                        nbytes = N * K + 2 * N + 2 * K + 2 * N
                        rec = {"path": name, "N": N, "K": K, "rpw": rpw, "wk": wk, "g": g,
                               "us": round(us, 3), "GBps": round(nbytes / us / 1e3, 1),
                               "err": err}
                        res.append(rec)
                        print(json.dumps(rec), flush=True)
            _lib.call("tao_tune_int8_gemv", 0, 0, 0)
            best = min(res, key=lambda r: r["us"])
            print(json.dumps({"BEST": best}), flush=True)
        del ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
