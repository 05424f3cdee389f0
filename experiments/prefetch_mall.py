"""Experiment: does reading the NEXT linear's weights on a side stream (default-policy loads, so
they land in the 256 MB MALL) while the current GEMV runs make the decode step faster? Llama-3-8B
int4 g32 linears (32 x {wqkv, wo, w1||w3, w2} + head, M = 1, distinct weights), one HIP graph per
variant: the 129 GEMVs in stream order, optionally with prefetch(j + 1) on a second stream after
GEMV j - 1 (so it overlaps GEMV j). ms per step, alternated, 3 rounds. One JSON line per
(variant, round).

    hipcc --offload-arch=gfx950 -O3 -shared -fPIC -o experiments/build/libprefetch.so \
      experiments/prefetch_mall.hip
    PYTHONPATH=torchao-fork_amd python experiments/prefetch_mall.py
"""
import ctypes
import json
import os

import torch

import torchao  # noqa: F401  (registers torch.ops.torchao)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pf = ctypes.CDLL(os.path.join(ROOT, "experiments", "build", "libprefetch.so"))
pf.prefetch_launch.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p,
                               ctypes.c_void_p]
DEV = "cuda"
G = 32


def weights():
    shapes = []
    for _ in range(32):
        shapes += [(6144, 4096), (4096, 4096), (28672, 4096), (4096, 14336)]
    shapes.append((128256, 4096))
    ws = []
    for N, K in shapes:
        packed = torch.randint(-2**31, 2**31 - 1, (N, K // 8), dtype=torch.int32, device=DEV)
        sz = (torch.rand(N, K // G, 2, device=DEV) * 0.01).to(torch.bfloat16)
        ws.append((packed, sz))
    return ws


def main():
    ws = weights()
    xs = {K: torch.randn(1, K, device=DEV, dtype=torch.bfloat16) for K in (4096, 14336)}
    sink = torch.zeros(1024, dtype=torch.int32, device=DEV)
    n = len(ws)

    def step(grid, ahead=1):
        s = torch.cuda.current_stream()
        p = torch.cuda.Stream() if grid else None
        evs = [torch.cuda.Event() for _ in range(n)]
        if p is not None:
            p.wait_stream(s)
        for j in range(n):
            packed, sz = ws[j]
            torch.ops.torchao.int4_weight_only_linear(xs[packed.shape[1] * 8], packed, sz, G)
            evs[j].record(s)
            if p is not None and j + ahead < n:
                with torch.cuda.stream(p):
                    if j >= 1:
                        p.wait_event(evs[j - 1])
                    nxt, nsz = ws[j + ahead]
                    for t in (nxt, nsz):
                        assert pf.prefetch_launch(t.data_ptr(), t.numel() * t.element_size(),
                                                  grid, sink.data_ptr(), p.cuda_stream) == 0
        if p is not None:
            s.wait_stream(p)

    variants = {"plain": (0, 1), "pf16": (16, 1), "pf64": (64, 1), "pf256": (256, 1),
                "pf64_ahead2": (64, 2)}
    graphs = {}
    for name, (grid, ahead) in variants.items():
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            step(grid, ahead)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                step(grid, ahead)
        torch.cuda.current_stream().wait_stream(s)
        graphs[name] = g
    torch.cuda.synchronize()
    for rnd in range(3):
        for name, g in graphs.items():
            for _ in range(3):
                g.replay()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                g.replay()
            e1.record()
            e1.synchronize()
            print(json.dumps({"variant": name, "round": rnd,
                              "ms_per_step": round(e0.elapsed_time(e1) / 20, 4)}), flush=True)


if __name__ == "__main__":
    main()
