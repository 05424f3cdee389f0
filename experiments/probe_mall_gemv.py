"""How much faster is an M = 1 int4 GEMV whose weights sit in the MALL (Infinity Cache, 256 MiB)
than one reading them from HBM? One graph of L launches cycling over C weight copies: C large
(footprint far past the MALL: every byte from HBM, as in the decode step) vs C small enough that
the copies stay in the MALL but not in the L2s. µs per launch from HIP events on the replay stream.

    PYTHONPATH=torchao-fork_amd python experiments/probe_mall_gemv.py
"""
import json

import torch

DEV = "cuda"


def weights(N, K, C, g=32):
    ws = []
    for _ in range(C):
        packed = torch.randint(-2**31, 2**31 - 1, (N, K // 8), dtype=torch.int32, device=DEV)
        sz = (torch.rand(N, K // g, 2, device=DEV) * 0.01).to(torch.bfloat16)
        ws.append((packed, sz))
    return ws


def time_graph(fn, L, reps=20):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for i in range(L):
            fn(i)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for i in range(L):
                fn(i)
    torch.cuda.current_stream().wait_stream(s)
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps / L


def main():
    import torchao  # noqa: F401
    K = 4096
    for N, K, c_cold, c_mall in ((4096, 4096, 64, 8), (6144, 4096, 48, 8), (28672, 4096, 8, 3),
                                 (4096, 14336, 16, 6)):
        x = torch.randn(1, K, device=DEV, dtype=torch.bfloat16)
        mb = N * K / 2 / 1e6
        for C in (c_cold, c_mall):
            ws = weights(N, K, C)
            L = max(C, 32)

            def fn(i):
                p, sz = ws[i % C]
                torch.ops.torchao.int4_weight_only_linear(x, p, sz, 32)

            us = time_graph(fn, L)
            print(json.dumps({"N": N, "K": K, "copies": C, "footprint_MB": round(C * mb * 1.125, 1),
                              "us_per_launch": round(us, 3),
                              "GBps": round(mb * 1.125 * 1e6 / (us * 1e-6) / 1e9, 1)}), flush=True)
            del ws
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
