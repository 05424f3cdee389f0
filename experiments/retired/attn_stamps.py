"""Per-workgroup timeline of the single-pass decode attention (TAO_ATTN_STAMPS=1 build,
experiments/build/libastamps.so via TORCHAO_MI355X_LIB): Llama-3-8B geometry (32 q heads, 8 kv
heads, D 128, cache 328 or 1024 rows), a HIP graph of 32 launches over distinct caches replayed
back to back; stamps of the last launch: first instruction, q landed, key loop done (wave 0),
end.

    TORCHAO_MI355X_LIB=experiments/build/libastamps.so python experiments/attn_stamps.py
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
from torchao._models.llama import kernels  # noqa: E402

lib = _lib.lib()
lib.tao_debug_attn_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]


def main():
    dev = torch.device("cuda")
    for T, p in ((512, 300), (1024, 900)):
        qs = [torch.randn(1, 32, 1, 128, device=dev, dtype=torch.bfloat16) for _ in range(32)]
        kcs = [torch.randn(1, 8, T, 128, device=dev, dtype=torch.bfloat16) for _ in range(32)]
        vcs = [torch.randn(1, 8, T, 128, device=dev, dtype=torch.bfloat16) for _ in range(32)]
        pos = torch.tensor([p], device=dev)
        s = torch.cuda.Stream()

        def run():
            for q, k, v in zip(qs, kcs, vcs):
                kernels.attn_decode(q, k, v, pos, 128 ** -0.5)

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
        per = e0.elapsed_time(e1) * 1e3 / 10 / 32
        buf = np.zeros(1024 * 4, dtype=np.uint64)
        assert lib.tao_debug_attn_stamps(buf.ctypes.data, 1024) == 0
        st = buf.reshape(1024, 4)
        st = st[st[:, 0] > 0].astype(np.int64)
        us = lambda a: a / 100.0  # noqa: E731
        e = st[:, 0].min()
        med = lambda a: round(float(us(np.median(a))), 2)  # noqa: E731
        print(json.dumps({"T": T, "pos": p, "us_per_launch_graph": round(per, 3),
                          "workgroups": int(len(st)),
                          "span_us": round(float(us(st[:, 3].max() - e)), 2),
                          "start_spread_us": round(float(us(st[:, 0].max() - e)), 2),
                          "q_landed_us": med(st[:, 1] - st[:, 0]),
                          "key_loop_us": med(st[:, 2] - st[:, 1]),
                          "merge_us": med(st[:, 3] - st[:, 2])}), flush=True)
        del g


if __name__ == "__main__":
    main()
