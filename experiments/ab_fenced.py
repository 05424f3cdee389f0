"""Fenced vs fence-free split-K hand-off: kernel us of every split-K launch the
routing makes at the Llama-3 8B / 70B prefill shapes (M = 16 .. 512; the shape table and the
heuristic decide the split), timed with tao_tune_splitk_fenced 0 and 1 alternately (A/B/A/B),
dispatch-packet events, weights rotated past the MALL. Outputs compared bit for bit.

    python experiments/ab_fenced.py [--out gpurun_out/r4_ab_fenced.jsonl]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "torchao-fork_amd"))
import torch  # noqa: E402

import torchao  # noqa: E402,F401
from torchao import _lib  # noqa: E402

DEV = "cuda"


def med(v):
    v = sorted(v)
    return v[len(v) // 2]


def timed(fn, copies, reps=20):
    for c in range(copies):
        fn(c)
    torch.cuda.synchronize()
    with _lib.KernelTimer(reps * 4) as kt:
        for i in range(reps):
            fn(i % copies)
    torch.cuda.synchronize()
    return med(kt.durations_ms) * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "r4_ab_fenced.jsonl"))
    args = ap.parse_args()
    out = open(args.out, "a")
    gen = torch.Generator(device=DEV).manual_seed(0)
    shapes = [(N, K) for N, K in ((6144, 4096), (4096, 4096), (28672, 4096), (4096, 14336),
                                  (10240, 8192), (8192, 8192), (8192, 28672))]
    for (N, K) in shapes:
        copies = max(2, int(256e6 // (N * K // 2)))
        w4 = []
        for _ in range(copies):
            q = torch.randint(0, 16, (N, K), dtype=torch.int32, device=DEV, generator=gen)
            sz = (torch.rand(N, K // 32, 2, device=DEV, generator=gen) * 0.02).to(torch.bfloat16)
            w4.append((torch.ops.torchao.int4_pack(q), sz))
            del q
        wq8 = [torch.randint(-127, 128, (N, K), dtype=torch.int8, device=DEV, generator=gen)
               for _ in range(max(2, copies // 2))]
        ws8 = (torch.rand(N, device=DEV, generator=gen) * 0.01 + 1e-3).to(torch.bfloat16)
        for M in (16, 32, 64, 128, 256, 512):
            x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16, generator=gen)
            xq, xs = torch.ops.torchao.int8_quantize_per_token(x)
            cases = {
                "int4": (lambda c: torch.ops.torchao.int4_weight_only_linear(
                    x, w4[c][0], w4[c][1], 32, None), copies),
                "int8dyn": (lambda c: torch.ops.torchao.int8_scaled_mm(
                    xq, xs, wq8[c], ws8, None), len(wq8)),
            }
            for path, (fn, cp) in cases.items():
                res = {}
                outs = {}
                for rnd in range(2):
                    for fenced in (0, 1):
                        _lib.call("tao_tune_splitk_fenced", fenced)
                        res.setdefault(fenced, []).append(timed(fn, cp))
                        outs[fenced] = fn(0).clone()
                _lib.call("tao_tune_reset")
                a, b = min(res[0]), min(res[1])
                rec = {"path": path, "M": M, "N": N, "K": K, "fence_free_us": round(a, 2),
                       "fenced_us": round(b, 2), "cost": round(b / a - 1, 4),
                       "bit_identical": bool(torch.equal(outs[0], outs[1]))}
                print(json.dumps(rec), flush=True)
                out.write(json.dumps(rec) + "\n")
        del w4, wq8
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
