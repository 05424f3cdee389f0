"""Per shape, graph wall time per launch of the int4 GEMV against a pure 16-B streaming read of
the same algorithmic bytes (block 512, one load per thread: the best read variant of
probe_graph_read.py), R launches per graph over rotated copies (> 512 MB, past the MALL).
Usage: python experiments/probe_graph_shapes.py [--tune rpw wk g occ]"""

import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "torchao-fork_amd"))
import torch  # noqa: E402

import bench  # noqa: E402
import torchao  # noqa: E402,F401
from torchao import _lib  # noqa: E402

probe = ctypes.CDLL(os.path.join(ROOT, "experiments", "libprobe.so"))
probe.probe_read_launch.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int,
                                    ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]


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
    t0 = time.perf_counter()
    for _ in range(reps):
        g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps / R * 1e6


def main():
    shapes = [(6144, 4096), (4096, 4096), (28672, 4096), (4096, 14336), (128256, 4096)]
    if len(sys.argv) > 1 and sys.argv[1] == "--shapes":
        shapes = [tuple(int(v) for v in s.split("x")) for s in sys.argv[2:]]
    dev = torch.device("cuda")
    lib = _lib.lib()
    out = torch.zeros(1024, dtype=torch.int32, device=dev)
    g = 32
    for N, K in shapes:
        nbytes = bench.int4_alg_bytes(N, K, g)
        copies = max(4, int(600e6 // nbytes) + 1)
        R = max(copies, 32)
        ws = []
        for _ in range(copies):
            p = torch.randint(-2**31, 2**31 - 1, (N, K // 8), dtype=torch.int32, device=dev)
            sz = (torch.rand(N, K // g, 2, device=dev) * 0.01).to(torch.bfloat16)
            ws.append((p, sz))
        x = torch.randn(1, K, device=dev, dtype=torch.bfloat16)
        y = torch.empty(1, N, device=dev, dtype=torch.bfloat16)
        u = 16 * 512
        rb = (nbytes + u - 1) // u * u
        rbufs = [torch.empty(rb, dtype=torch.uint8, device=dev) for _ in range(copies)]

        def gemv():
            st = torch.cuda.current_stream().cuda_stream
            for i in range(R):
                p, sz = ws[i % copies]
                lib.tao_int4wo_linear_bf16(x.data_ptr(), p.data_ptr(), sz.data_ptr(), None,
                                           y.data_ptr(), 1, N, K, g, st)

        def read():
            st = torch.cuda.current_stream().cuda_stream
            for i in range(R):
                probe.probe_read_launch(rbufs[i % copies].data_ptr(), rb, 512, 1, 1,
                                        out.data_ptr(), st)

        tg, tr = graph_us(gemv, R), graph_us(read, R)
        print(json.dumps({"N": N, "K": K, "bytes": nbytes, "gemv_us": round(tg, 3),
                          "read_us": round(tr, 3), "gemv_GBps": round(nbytes / tg / 1e3, 1),
                          "read_GBps": round(nbytes / tr / 1e3, 1),
                          "gemv_over_read": round(tg / tr, 3)}), flush=True)
        del ws, rbufs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
