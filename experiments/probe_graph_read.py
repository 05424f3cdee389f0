"""What a launch-per-linear design can reach on this chip: the bench step's 129 launches
(Llama-3-8B int4 g32 linears, M = 1) replayed from one HIP graph as PURE 16-B streaming reads of
the same byte counts (each launch its own buffer, 4.7 GB per step, so nothing is served by the
Infinity Cache), against the bench's GEMV step graph. Prints one JSON line per read variant.
Usage: python experiments/probe_graph_read.py  (needs experiments/libprobe.so:
hipcc -O3 --offload-arch=gfx950 -shared -fPIC experiments/probe.hip -o experiments/libprobe.so)"""

import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402

probe = ctypes.CDLL(os.path.join(ROOT, "experiments", "libprobe.so"))
probe.probe_read_launch.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int,
                                    ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]


def graph_ms(fn, reps=10):
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
        with torch.cuda.graph(g, stream=s):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


def main():
    dev = torch.device("cuda")
    plan = bench.llama_linears(bench.LLAMA3_8B)
    sizes = [bench.int4_alg_bytes(N, K, 32) for (_, N, K) in plan]
    total = sum(sizes)
    unit = 16 * 512 * 16
    bufs = [torch.empty((b + unit - 1) // unit * unit, dtype=torch.uint8, device=dev) for b in sizes]
    for b in bufs:
        b.fill_(7)
    out = torch.zeros(1024, dtype=torch.int32, device=dev)
    for block in (256, 512):
        for L in (1, 2, 4, 8, 16):
            def run():
                st = torch.cuda.current_stream().cuda_stream
                for b, n in zip(bufs, sizes):
                    u = 16 * block * L
                    probe.probe_read_launch(b.data_ptr(), (n + u - 1) // u * u, block, L, 1,
                                            out.data_ptr(), st)
            ms = graph_ms(run)
            print(json.dumps({"probe": "graph_read_step", "launches": len(plan), "block": block,
                              "L": L, "nt": 1, "ms_per_step": round(ms, 4),
                              "GBps_alg": round(total / ms / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
