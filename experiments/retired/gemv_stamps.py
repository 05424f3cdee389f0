"""Per-workgroup timeline of the M = 1 int4 GEMV (TAO_GEMV_STAMPS=1 build,
experiments/build/libgstamps.so via TORCHAO_MI355X_LIB): a HIP graph of 32 launches over
distinct weights replayed back to back; the last launch's stamps (s_memrealtime, 10 ns) of
every workgroup's wave 0: first instruction, slices done, end.

    TORCHAO_MI355X_LIB=experiments/build/libgstamps.so python experiments/gemv_stamps.py

Also per shape: end-time percentiles, the most workgroups running at once, and a pure 16-B read
of the same bytes (tao_hbm_read_probe) replayed the same way, for the per-launch gap to it.
"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "torchao-fork_amd"))
from torchao import _lib  # noqa: E402

lib = _lib.lib()
lib.tao_debug_gemv_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
NB = 65536
G = 32


def main():
    dev = torch.device("cuda")
    for N, K in ((4096, 4096), (6144, 4096), (28672, 4096), (4096, 14336)):
        ws = []
        for i in range(32):
            q = torch.randint(0, 16, (N, K), dtype=torch.int32, device=dev)
            sz = (torch.rand(N, K // G, 2, device=dev) * 0.02).to(torch.bfloat16)
            ws.append((torch.ops.torchao.int4_pack(q), sz))
        x = torch.randn(1, K, device=dev, dtype=torch.bfloat16)
        y = torch.empty(N, device=dev, dtype=torch.bfloat16)
        s = torch.cuda.Stream()

        def run():
            sp = torch.cuda.current_stream().cuda_stream
            for p, z in ws:
                assert lib.tao_int4wo_linear_bf16(x.data_ptr(), p.data_ptr(), z.data_ptr(), None,
                                                  y.data_ptr(), 1, N, K, G, sp) == 0

        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            run()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                run()
        torch.cuda.current_stream().wait_stream(s)
        for _ in range(3):
            g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        per_launch = e0.elapsed_time(e1) * 1e3 / 10 / 32
        nbytes = (N * K // 2 + N * (K // G) * 4 + 8191) // 8192 * 8192
        rb = [torch.empty(nbytes, dtype=torch.uint8, device=dev).fill_(7) for _ in range(32)]
        sink = torch.zeros(1024, dtype=torch.int32, device=dev)

        def rrun():
            sp = torch.cuda.current_stream().cuda_stream
            for b in rb:
                assert lib.tao_hbm_read_probe(b.data_ptr(), nbytes, sink.data_ptr(), sp) == 0
        with torch.cuda.stream(s):
            rrun()
            gr = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gr, stream=s):
                rrun()
        torch.cuda.current_stream().wait_stream(s)
        for _ in range(3):
            gr.replay()
        e0.record()
        for _ in range(10):
            gr.replay()
        e1.record()
        torch.cuda.synchronize()
        read_per_launch = e0.elapsed_time(e1) * 1e3 / 10 / 32
        del gr, rb
        # the GEMV graph once more, so the stamps are the GEMV's
        g.replay()
        torch.cuda.synchronize()
        buf = np.zeros(NB * 4, dtype=np.uint64)
        assert lib.tao_debug_gemv_stamps(buf.ctypes.data, NB) == 0
        st = buf.reshape(NB, 4)
        st = st[st[:, 0] > 0].astype(np.int64)
        us = lambda a: a / 100.0  # noqa: E731
        e = st[:, 0].min()
        rec = {"N": N, "K": K, "us_per_launch_graph": round(per_launch, 3),
               "workgroups": int(len(st)),
               "span_us": round(float(us(st[:, 2].max() - e)), 2),
               "entry_spread_us": round(float(us(st[:, 0].max() - e)), 2),
               "entry_p50_us": round(float(us(np.median(st[:, 0] - e))), 2),
               "loads_compute_us": [round(float(us(np.median(st[:, 1] - st[:, 0]))), 2),
                                    round(float(us((st[:, 1] - st[:, 0]).max())), 2)],
               "tail_us": [round(float(us(np.median(st[:, 2] - st[:, 1]))), 2),
                           round(float(us((st[:, 2] - st[:, 1]).max())), 2)],
               "last_end_minus_p90_end_us": round(float(us(st[:, 2].max() - np.percentile(st[:, 2], 90))), 2),
               "end_pct_us": [round(float(us(np.percentile(st[:, 2], q) - e)), 2)
                              for q in (10, 50, 90, 99)],
               "max_concurrent_wgs": int(max(
                   ((st[:, 0] <= t) & (st[:, 2] > t)).sum() for t in np.linspace(e, st[:, 2].max(), 200))),
               "pure_read_us_per_launch": round(read_per_launch, 3),
               "bytes": nbytes}
        print(json.dumps(rec), flush=True)
        del g, ws


if __name__ == "__main__":
    main()
