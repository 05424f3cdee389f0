"""Is the ~4 us duration of tiny kernels real? Compare, in one process:
  (a) wall time per launch of R back-to-back launches replayed from a HIP graph,
  (b) per-launch dispatch-event durations (tao_profile_*),
for an empty kernel and for the int4 GEMV at 4096x4096 / 14336x4096 (weights rotated over
> 256 MiB). Run under rocprofv3 --kernel-trace --stats to get (c) the profiler's durations."""

import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "torchao-fork_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import torchao  # noqa: E402,F401
from torchao import _lib  # noqa: E402

probe = ctypes.CDLL(os.path.join(ROOT, "experiments", "libprobe.so"))
probe.probe_empty_launch.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p]


def graph_time(fn, reps=5):
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
        with torch.cuda.graph(g, stream=s):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        g.replay()
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t0)
    return best


def main():
    R = 200
    cur = lambda: torch.cuda.current_stream().cuda_stream
    t = graph_time(lambda: [probe.probe_empty_launch(256, 256, cur()) for _ in range(R)])
    print(json.dumps({"what": "empty graph wall per launch", "us": round(t / R * 1e6, 3)}))

    lib = _lib.lib()
    for (N, K) in [(4096, 4096), (14336, 4096), (4096, 14336)]:
        g = 32
        copies = max(8, int(400e6 // (N * K // 2)))
        ws = []
        for i in range(copies):
            q = torch.randint(0, 16, (N, K), dtype=torch.int32, device="cuda")
            p = torch.ops.torchao.int4_pack(q)
            sz = (torch.rand(N, K // g, 2, device="cuda") * 0.01).to(torch.bfloat16)
            ws.append((p, sz))
            del q
        x = torch.randn(1, K, device="cuda", dtype=torch.bfloat16)
        y = torch.empty(1, N, device="cuda", dtype=torch.bfloat16)

        def run(n):
            for i in range(n):
                p, sz = ws[i % copies]
                lib.tao_int4wo_linear_bf16(x.data_ptr(), p.data_ptr(), sz.data_ptr(), None,
                                           y.data_ptr(), 1, N, K, g, cur())

        t = graph_time(lambda: run(R))
        with _lib.KernelTimer(R) as kt:
            run(R)
        d = sorted(kt.durations_ms)
        med = d[len(d) // 2]
        print(json.dumps({"what": f"int4 gemv {N}x{K}", "graph_wall_us_per_launch": round(t / R * 1e6, 3),
                          "event_us_median": round(med * 1e3, 3), "event_us_min": round(d[0] * 1e3, 3)}))
        del ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
