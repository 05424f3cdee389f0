"""Decode-attention launch cost per kernel (tao_tune_attn modes), Llama-3-8B heads (32 q, 8 kv,
D 128), B = 1: 32 launches over 32 distinct layer caches (as one decoded token runs them) captured
in one HIP graph; µs per launch from HIP events on the replay stream, and the kernels' own
durations (dispatch-packet events, tao_profile_*) from one eager pass. One JSON line per
(mode, keys) to stdout.

    python experiments/attn_time.py [--modes 0,2] [--keys 128,200,256,300,328,512,900]
"""
import argparse
import json
import math
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "torchao-fork_amd"))

from torchao import _lib  # noqa: E402
from torchao._models.llama import kernels  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--modes", default="0,2")
    ap.add_argument("--keys", default="128,200,256,300,328,512,900")
    ap.add_argument("--T", type=int, default=1024)
    ap.add_argument("--reps", type=int, default=50)
    a = ap.parse_args()
    dev = torch.device("cuda")
    H, Hkv, D, T, NL = 32, 8, 128, a.T, 32
    gen = torch.Generator(device=dev).manual_seed(0)
    kcs = [torch.randn(1, Hkv, T, D, device=dev, dtype=torch.bfloat16, generator=gen) for _ in range(NL)]
    vcs = [torch.randn(1, Hkv, T, D, device=dev, dtype=torch.bfloat16, generator=gen) for _ in range(NL)]
    q = torch.randn(1, H, 1, D, device=dev, dtype=torch.bfloat16, generator=gen)
    pos = torch.zeros(1, dtype=torch.int64, device=dev)
    s = torch.cuda.Stream(dev)
    for L in [int(x) for x in a.keys.split(",")]:
        pos.fill_(L - 1)
        for mode in [int(m) for m in a.modes.split(",")]:
            _lib.call("tao_tune_attn", mode)
            outs = [None] * NL

            def step():
                for i in range(NL):
                    outs[i] = kernels.attn_decode(q, kcs[i], vcs[i], pos, 1 / math.sqrt(D))

            s.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(s):
                step()
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=s):
                    step()
                g.replay()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                for _ in range(a.reps):
                    g.replay()
                e1.record(s)
            e1.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / a.reps / NL
            torch.cuda.current_stream(dev).wait_stream(s)
            with _lib.KernelTimer(4 * NL) as kt:
                step()
            torch.cuda.synchronize()
            d = sorted(kt.durations_ms)
            ref = torch.nn.functional.scaled_dot_product_attention(
                q.float(), kcs[0][:, :, :L].float(), vcs[0][:, :, :L].float(), enable_gqa=True)
            err = float((outs[0].float().reshape(-1) - ref.reshape(-1)).abs().max())
            print(json.dumps({"mode": mode, "keys": L, "T": T, "us_per_launch_graph": round(us, 3),
                              "kernel_us_median": round(d[len(d) // 2] * 1e3, 3),
                              "kernels_per_call": len(d) // NL, "max_abs_err_vs_fp32": round(err, 5)}),
                  flush=True)
            del g
    _lib.call("tao_tune_attn", 0)


if __name__ == "__main__":
    main()
