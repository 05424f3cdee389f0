"""Occupancy cap of the int4 M = 1 GEMV by reserved LDS (tao_tune_int4_lds): per shape, 32
launches over distinct weights (past the MALL) in one HIP graph, µs per launch from HIP events on
the replay stream; settings interleaved and repeated (--passes); outputs checked bit-identical to
the built-in launch (same launch shape, only residency changes). One JSON line per (shape,
setting, pass).

    python experiments/ab_gemv_lds.py [--lds 0,27000,40960,54000,81920] [--passes 2]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "torchao-fork_amd"))

from torchao import _lib  # noqa: E402

SHAPES = [(28672, 4096), (4096, 14336), (6144, 4096), (4096, 4096), (128256, 4096)]


def graph_us(fn, n, reps=20):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            fn()
        g.replay()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(reps):
            g.replay()
        e1.record(s)
    e1.synchronize()
    torch.cuda.current_stream().wait_stream(s)
    return e0.elapsed_time(e1) * 1e3 / reps / n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lds", default="0,20480,27000,32768,40960,54000,81920")
    ap.add_argument("--passes", type=int, default=2)
    ap.add_argument("--shapes", default="")
    a = ap.parse_args()
    dev = torch.device("cuda")
    lib = _lib.lib()
    settings = [int(v) for v in a.lds.split(",")]
    shapes = ([tuple(int(v) for v in t.split("x")) for t in a.shapes.split(",")] if a.shapes
              else SHAPES)
    gen = torch.Generator(device=dev).manual_seed(0)
    for N, K in shapes:
        copies = max(2, min(32, (320 << 20) // (N * K // 2)))
        ws = []
        for _ in range(copies):
            w = (torch.randn(N, K, device=dev, generator=gen) * 0.02).to(torch.bfloat16)
            ws.append(torch.ops.torchao.int4_quantize_pack(w, 32, 1e-6))
            del w
        x = torch.randn(1, K, device=dev, dtype=torch.bfloat16, generator=gen)
        ys = [torch.empty(1, N, device=dev, dtype=torch.bfloat16) for _ in ws]

        def run():
            sp = torch.cuda.current_stream().cuda_stream
            for (p, z), y in zip(ws, ys):
                rc = lib.tao_int4wo_linear_bf16(x.data_ptr(), p.data_ptr(), z.data_ptr(), None,
                                                y.data_ptr(), 1, N, K, 32, sp)
                if rc:
                    raise RuntimeError(lib.tao_last_error().decode())

        ref = None
        for ps in range(a.passes):
            for lds in settings:
                _lib.call("tao_tune_int4_lds", lds)
                us = graph_us(run, copies)
                run()
                torch.cuda.synchronize()
                out = torch.stack([y.clone() for y in ys])
                if ref is None:
                    ref = out
                print(json.dumps({"N": N, "K": K, "lds": lds, "pass": ps, "us": round(us, 3),
                                  "launches": copies, "bit_identical": bool(torch.equal(out, ref))}),
                      flush=True)
        _lib.call("tao_tune_int4_lds", 0)
        del ws, ys


if __name__ == "__main__":
    main()
