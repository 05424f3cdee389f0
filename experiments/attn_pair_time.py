"""Decode attention + wo (+ residual) per layer, Llama-3-8B heads (32 q, 8 kv, D 128), B = 1:
32 layers (distinct caches and distinct int4 wo weights, as one decoded token runs them) in one
HIP graph, µs per layer from HIP events on the replay stream. Variants:
  onepass    tao_attn_decode_bf16 (one workgroup per head) -> int4 linear with bias = residual
  splitS     tao_attn_decode_split_bf16 (S key ranges per head) -> tao_int4wo_attn_out_bf16
  attn_only  / split_only: the attention launches alone (32 per graph)
One JSON line per (variant, keys) to stdout.

    python experiments/attn_pair_time.py [--keys 128,328,512,900] [--splits 2,4]
"""
import argparse
import json
import math
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "torchao-fork_amd"))

from torchao._models.llama import kernels  # noqa: E402


def graph_us(fn, reps, n, dev):
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
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
    torch.cuda.current_stream(dev).wait_stream(s)
    return e0.elapsed_time(e1) * 1e3 / reps / n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--keys", default="128,328,512,900")
    ap.add_argument("--splits", default="2,4")
    ap.add_argument("--T", type=int, default=1024)
    ap.add_argument("--reps", type=int, default=50)
    a = ap.parse_args()
    dev = torch.device("cuda")
    H, Hkv, D, T, NL, g = 32, 8, 128, a.T, 32, 32
    N = K = H * D
    gen = torch.Generator(device=dev).manual_seed(0)
    kcs = [torch.randn(1, Hkv, T, D, device=dev, dtype=torch.bfloat16, generator=gen) for _ in range(NL)]
    vcs = [torch.randn(1, Hkv, T, D, device=dev, dtype=torch.bfloat16, generator=gen) for _ in range(NL)]
    wos = []
    for _ in range(NL):
        w = (torch.randn(N, K, device=dev, generator=gen) / math.sqrt(K)).to(torch.bfloat16)
        wos.append(torch.ops.torchao.int4_quantize_pack(w, g, 1e-6))
    q = torch.randn(1, H, 1, D, device=dev, dtype=torch.bfloat16, generator=gen)
    res = torch.randn(1, 1, N, device=dev, dtype=torch.bfloat16, generator=gen)
    pos = torch.zeros(1, dtype=torch.int64, device=dev)
    scale = 1 / math.sqrt(D)
    outs = [None] * NL

    def onepass(with_wo=True):
        def f():
            for i in range(NL):
                y = kernels.attn_decode(q, kcs[i], vcs[i], pos, scale)
                if with_wo:
                    y = torch.ops.torchao.int4_weight_only_linear(y, wos[i][0], wos[i][1], g,
                                                                  res.reshape(-1))
                outs[i] = y
        return f

    def split(S, with_wo=True):
        def f():
            for i in range(NL):
                part = kernels.attn_decode_split(q, kcs[i], vcs[i], pos, scale, S)
                outs[i] = (kernels.int4_attn_out(part, H, wos[i][0], wos[i][1], g, residual=res)
                           if with_wo else part)
        return f

    for L in [int(x) for x in a.keys.split(",")]:
        pos.fill_(L - 1)
        variants = [("onepass", onepass()), ("attn_only", onepass(False))]
        for S in [int(x) for x in a.splits.split(",")]:
            variants += [(f"split{S}", split(S)), (f"split{S}_only", split(S, False))]
        ref = None
        for name, fn in variants:
            us = graph_us(fn, a.reps, NL, dev)
            rec = {"variant": name, "keys": L, "T": T, "us_per_layer_graph": round(us, 3)}
            if not name.endswith("only"):
                fn()
                torch.cuda.synchronize()
                y = outs[0].float().reshape(-1)
                if ref is None:
                    ref = y
                else:
                    rec["rel_l2_vs_onepass"] = round(float((y - ref).norm() / ref.norm()), 6)
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
