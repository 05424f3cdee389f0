"""Side-stream weight prefetch experiment (see prefetch.hip). Prints JSON lines:
  * per shape: int4 GEMV kernel time with its weights cold (rotated past the MALL) vs hot
    (the same weights back to back, MALL-resident);
  * the bench.py step (129 GEMVs, Llama-3-8B shapes, one HIP graph) with and without a
    prefetcher on a second stream that streams linear i+1's weights while GEMV i runs.
Random packed bytes stand in for quantized weights (timing does not depend on the values)."""

import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "torchao-fork_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from bench import LLAMA3_8B, llama_linears  # noqa: E402
from torchao import _lib  # noqa: E402

pf = ctypes.CDLL(os.path.join(ROOT, "experiments", "libprefetch.so"))
pf.pf_launch.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int,
                         ctypes.c_void_p, ctypes.c_void_p]
lib = _lib.lib()
dev = torch.device("cuda")
G = 32


def weight(N, K):
    packed = torch.randint(-2**31, 2**31 - 1, (N, K // 8), dtype=torch.int32, device=dev)
    sz = (torch.rand(N, K // G, 2, device=dev) * 0.01).to(torch.bfloat16)
    return packed, sz


def gemv(x, packed, sz, y, N, K, stream):
    rc = lib.tao_int4wo_linear_bf16(x.data_ptr(), packed.data_ptr(), sz.data_ptr(), None,
                                    y.data_ptr(), 1, N, K, G, stream)
    assert rc == 0, lib.tao_last_error()


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else "all"
    lins = llama_linears(LLAMA3_8B)
    xs = {K: torch.randn(1, K, device=dev, dtype=torch.bfloat16) for _, _, K in lins}
    sink = torch.zeros(1024, dtype=torch.int32, device=dev)

    if which in ("all", "hot"):
        for N, K in [(6144, 4096), (4096, 4096), (28672, 4096), (4096, 14336), (128256, 4096)]:
            copies = max(2, int(600e6 // (N * K // 2)))
            ws = [weight(N, K) for _ in range(copies)]
            y = torch.empty(N, device=dev, dtype=torch.bfloat16)
            sp = torch.cuda.current_stream().cuda_stream
            reps = 40
            with _lib.KernelTimer(reps) as t:
                for r in range(reps):
                    p, s = ws[r % copies]
                    gemv(xs[K], p, s, y, N, K, sp)
            cold = statistics.median(t.durations_ms[4:]) * 1e3
            with _lib.KernelTimer(reps) as t:
                for r in range(reps):
                    gemv(xs[K], ws[0][0], ws[0][1], y, N, K, sp)
            hot = statistics.median(t.durations_ms[4:]) * 1e3
            # prefetch kernel alone on the cold copies (rate it can stream at)
            pft = {}
            for grid in (128, 256, 512, 1024):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for r in range(reps):
                    p, s = ws[r % copies]
                    pf.pf_launch(p.data_ptr(), p.numel() * 4, grid, 1, sink.data_ptr(), sp)
                e1.record()
                e1.synchronize()
                pft[grid] = round(e0.elapsed_time(e1) / reps * 1e3, 2)
            print(json.dumps({"shape": f"{N}x{K}", "cold_us": round(cold, 2),
                              "hot_us": round(hot, 2), "pf_wall_us_by_grid": pft}), flush=True)
            del ws
            torch.cuda.empty_cache()

    if which in ("all", "step"):
        plan = []
        for _, N, K in lins:
            p, s = weight(N, K)
            plan.append((N, K, p, s, torch.empty(N, device=dev, dtype=torch.bfloat16)))
        torch.cuda.synchronize()
        main_s, side_s = torch.cuda.Stream(), torch.cuda.Stream()
        n = len(plan)

        def capture(pf_cfg):
            g = torch.cuda.CUDAGraph()
            main_s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(main_s):
                for _ in range(2):
                    body(pf_cfg)
                with torch.cuda.graph(g, stream=main_s):
                    body(pf_cfg)
            torch.cuda.current_stream().wait_stream(main_s)
            torch.cuda.synchronize()
            return g

        def body(pf_cfg):
            ms = main_s.cuda_stream
            if pf_cfg is None:
                for (N, K, p, s, y) in plan:
                    gemv(xs[K], p, s, y, N, K, ms)
                return
            grid, pol, wait, ahead = pf_cfg
            ss = side_s.cuda_stream
            evP = [torch.cuda.Event() for _ in range(n)]
            evG = [torch.cuda.Event() for _ in range(n)]
            side_s.wait_stream(main_s)

            def prefetch(j):
                N, K, p, s, _ = plan[j]
                pf.pf_launch(p.data_ptr(), p.numel() * 4, grid, pol, sink.data_ptr(), ss)
                pf.pf_launch(s.data_ptr(), s.numel() * 2, max(grid // 8, 8), pol,
                             sink.data_ptr(), ss)
                evP[j].record(side_s)

            for j in range(min(ahead, n)):
                prefetch(j)
            for i in range(n):
                # the loader for linear i + ahead starts once GEMV i - 1 is done, so at most
                # `ahead` linears' weights are in flight beyond the running GEMV
                j = i + ahead
                if j < n:
                    if i >= 1:
                        side_s.wait_event(evG[i - 1])
                    prefetch(j)
                N, K, p, s, y = plan[i]
                if wait:
                    main_s.wait_event(evP[i])
                gemv(xs[K], p, s, y, N, K, ms)
                evG[i].record(main_s)
            main_s.wait_stream(side_s)

        def time_graph(g, reps=20):
            with torch.cuda.stream(main_s):
                g.replay()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(main_s)
                for _ in range(reps):
                    g.replay()
                e1.record(main_s)
            e1.synchronize()
            return e0.elapsed_time(e1) / reps

        bytes_step = sum(N * K // 2 + (K // G) * N * 4 for N, K, *_ in plan)
        cfgs = [None]
        for grid in (128, 256, 512):
            for pol in (0, 1):
                for wait in (True, False):
                    cfgs.append((grid, pol, wait, 1))
        cfgs += [(256, 0, True, 2), (256, 1, True, 2), None]
        for c in cfgs:
            g = capture(c)
            ms = min(time_graph(g) for _ in range(3))
            print(json.dumps({"step_cfg": c, "ms": round(ms, 4),
                              "GBps": round(bytes_step / (ms * 1e-3) / 1e9, 1),
                              "tok_s": round(1e3 / ms, 1)}), flush=True)
            del g


if __name__ == "__main__":
    main()
