"""Driver of experiments/probe_two_streams.hip (loads only, the decode GEMV's shape): us per
launch in a HIP graph of 32 launches over 32 distinct buffers (past the 256 MiB MALL), for the
two-array layout (the library's), one interleaved array, nibbles only and row-quad words; and a
pure 16-B read of the same bytes (tao_hbm_read_probe). One JSON line per (N, mode).

    PYTHONPATH=torchao-fork_amd python experiments/probe_two_streams.py
"""
import ctypes
import json
import os

import torch

from torchao import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
lib = ctypes.CDLL(os.path.join(ROOT, "experiments", "build", "libprobe2s.so"))
lib.probe2s_launch.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                               ctypes.c_void_p, ctypes.c_void_p]
tao = _lib.lib()
dev = torch.device("cuda")
COPIES = 32


def graph_us(launch):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        launch()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            launch()
    torch.cuda.current_stream().wait_stream(s)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = []
    for _ in range(3):
        e0.record()
        for _ in range(10):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        best.append(e0.elapsed_time(e1) * 1e3 / 10 / COPIES)
    return sorted(best)[1]


def main():
    sink = torch.zeros(1024, dtype=torch.int32, device=dev)
    for N in (4096, 28672):
        wb, sbytes = N * 2048, N * 512
        bufs = [torch.empty(wb + sbytes, dtype=torch.uint8, device=dev).fill_(3)
                for _ in range(COPIES)]
        for mode, name in ((0, "two arrays"), (1, "interleaved rows"), (2, "nibbles only"),
                           (3, "two arrays, row-quad words")):
            def launch(mode=mode):
                sp = torch.cuda.current_stream().cuda_stream
                for b in bufs:
                    p = b.data_ptr()
                    assert lib.probe2s_launch(mode, p, p + wb, N, sink.data_ptr(), sp) == 0
            us = graph_us(launch)
            nbytes = wb if mode == 2 else wb + sbytes
            print(json.dumps({"N": N, "K": 4096, "mode": mode, "layout": name, "bytes": nbytes,
                              "us_per_launch": round(us, 3),
                              "GBps": round(nbytes / us / 1e3, 1)}), flush=True)

        def rlaunch():
            sp = torch.cuda.current_stream().cuda_stream
            for b in bufs:
                assert tao.tao_hbm_read_probe(b.data_ptr(), wb + sbytes, sink.data_ptr(), sp) == 0
        us = graph_us(rlaunch)
        print(json.dumps({"N": N, "K": 4096, "mode": "pure read", "bytes": wb + sbytes,
                          "us_per_launch": round(us, 3),
                          "GBps": round((wb + sbytes) / us / 1e3, 1)}), flush=True)
        del bufs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
