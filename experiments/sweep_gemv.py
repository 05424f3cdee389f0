"""Sweep the int4 M=1 GEMV launch shape (tao_tune_int4_gemv) per weight shape.

For each (N, K): weights rotated over > 300 MB of copies (Infinity Cache defeated), one
dispatch-event timing per launch (KernelTimer), median over launches; each config's output is
checked against the default config (rel L2 < 1e-3). Prints JSON lines, best config last.
--graph: time instead by the wall time per launch of R back-to-back launches replayed from one
HIP graph (how bench.py and the decode harness run them; dispatch events floor at ~4 us and hide
differences between small shapes)."""

import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "torchao-fork_amd"))
import torch  # noqa: E402

import torchao  # noqa: E402,F401
from torchao import _lib  # noqa: E402

SHAPES = [(4096, 4096), (6144, 4096), (14336, 4096), (4096, 14336), (128256, 4096),
          (10240, 8192), (8192, 8192), (28672, 8192), (8192, 28672),
          (1280, 8192), (1024, 8192), (3584, 8192), (1024, 28672)]


def bytes_of(N, K, g=32):
    return N * K // 2 + (K // g) * N * 4 + K * 2 + N * 2


def graph_us(fn, R, reps=10):
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
        with torch.cuda.graph(g, stream=s):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    g.replay()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(3):
        t0 = time.perf_counter()
        for _ in range(reps):
            g.replay()
        torch.cuda.synchronize()
        best = min(best, (time.perf_counter() - t0) / reps / R * 1e6)
    return best


def main():
    args = sys.argv[1:]
    use_graph = "--graph" in args
    xlds = "--xlds" in args  # x staged in LDS per workgroup (tao_tune_int4_xlds 1)
    args = [a for a in args if a not in ("--graph", "--xlds")]
    shapes = SHAPES if not args else [tuple(map(int, s.split("x"))) for s in args]
    lib = _lib.lib()
    lib.tao_tune_int4_xlds(1 if xlds else 0)
    g = 32
    for (N, K) in shapes:
        S = (K // 32 + 63) // 64
        copies = max(4, min(64, int(400e6 // bytes_of(N, K))))
        ws = []
        for _ in range(copies):
            q = torch.randint(0, 16, (N, K), dtype=torch.int32, device="cuda")
            ws.append((torch.ops.torchao.int4_pack(q), (torch.rand(N, K // g, 2, device="cuda") * 0.02).to(torch.bfloat16)))
            del q
        x = torch.randn(1, K, device="cuda", dtype=torch.bfloat16)
        ys = torch.empty(1, N, device="cuda", dtype=torch.bfloat16)
        reps = max(copies, 48)

        def run(n):
            st = torch.cuda.current_stream().cuda_stream
            for i in range(n):
                p, sz = ws[i % copies]
                lib.tao_int4wo_linear_bf16(x.data_ptr(), p.data_ptr(), sz.data_ptr(), None,
                                           ys.data_ptr(), 1, N, K, g, st)

        lib.tao_tune_int4_gemv(0, 0, 0, 0)
        p, sz = ws[0]
        ref = torch.ops.torchao.int4_weight_only_linear(x, p, sz, g, None).float()
        results = []
        cands = []
        for rpw in ((2, 4) if xlds else (1, 2, 4, 8)):
            for occ in ((4, 8) if rpw == 4 else (0,)):
                for wk in sorted({w for w in (1, 2, 3, 4, 7, 8) if w <= S} | {min(S, 8)}):
                    for gg in (1, 2, 4, 8):
                        if wk * gg <= 8:
                            cands.append((rpw, wk, gg, occ))
        for (rpw, wk, gg, occ) in cands:
            if lib.tao_tune_int4_gemv(rpw, wk, gg, occ) != 0:
                continue
            y = torch.ops.torchao.int4_weight_only_linear(x, p, sz, g, None).float()
            err = float((y - ref).norm() / ref.norm())
            if use_graph:
                us = graph_us(lambda: run(reps), reps)
            else:
                run(4)
                with _lib.KernelTimer(reps) as kt:
                    run(reps)
                d = sorted(kt.durations_ms)
                us = d[len(d) // 2] * 1e3
            rec = {"timing": "graph" if use_graph else "events", "xlds": xlds, "N": N, "K": K, "rpw": rpw, "wk": wk, "g": gg, "occ": occ, "us": round(us, 3),
                   "GBps": round(bytes_of(N, K) / us / 1e3, 1), "err": round(err, 6)}
            results.append(rec)
            print(json.dumps(rec), flush=True)
        lib.tao_tune_int4_gemv(0, 0, 0, 0)
        ok = [r for r in results if r["err"] < 1e-3]
        best = min(ok, key=lambda r: r["us"])
        print(json.dumps({"BEST": best}), flush=True)
        del ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
