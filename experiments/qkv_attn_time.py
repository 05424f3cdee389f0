"""Decode RMSNorm -> wqkv -> RoPE + KV -> attention per layer, Llama-3-8B (dim 4096, 32 q / 8 kv
heads, D 128, int4 g 32), B = 1: 32 layers (distinct wqkv weights and caches, as one decoded
token runs them) in one HIP graph, us per layer from HIP events on the replay stream. Variants:
  two        tao_int4wo_decode_bf16 (rope_kv epilogue) -> tao_attn_decode_bf16 (two launches)
  fusedS     tao_int4wo_qkv_attn_bf16 with S key ranges per head (one launch)
  gemv_only  the wqkv launch alone (what the attention adds on top of it)
One JSON line per (variant, keys).

    PYTHONPATH=torchao-fork_amd python experiments/qkv_attn_time.py [--keys 128,328,512,900]
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
from torchao._models.llama.model import ModelArgs, _rope_freqs  # noqa: E402


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
        ts = []
        for _ in range(3):
            e0.record(s)
            for _ in range(reps):
                g.replay()
            e1.record(s)
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3 / reps / n)
    torch.cuda.current_stream(dev).wait_stream(s)
    return sorted(ts)[1]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--keys", default="128,328,512,900")
    ap.add_argument("--T", type=int, default=1024)
    ap.add_argument("--reps", type=int, default=30)
    a = ap.parse_args()
    dev = torch.device("cuda")
    H, Hkv, D, T, NL, g, dim = 32, 8, 128, a.T, 32, 32, 4096
    N = (H + 2 * Hkv) * D
    gen = torch.Generator(device=dev).manual_seed(0)
    kcs = [torch.randn(1, Hkv, T, D, device=dev, dtype=torch.bfloat16, generator=gen) for _ in range(NL)]
    vcs = [torch.randn(1, Hkv, T, D, device=dev, dtype=torch.bfloat16, generator=gen) for _ in range(NL)]
    ws = []
    for _ in range(NL):
        w = (torch.randn(N, dim, device=dev, generator=gen) / math.sqrt(dim)).to(torch.bfloat16)
        ws.append(torch.ops.torchao.int4_quantize_pack(w, g, 1e-6))
    nw = (torch.rand(dim, device=dev, generator=gen) + 0.5).to(torch.bfloat16)
    x = torch.randn(1, 1, dim, device=dev, dtype=torch.bfloat16, generator=gen)
    cfg = ModelArgs(n_layer=1, n_head=H, n_local_heads=Hkv, dim=dim, rope_base=500000)
    freqs = _rope_freqs(cfg, T).to(dev)
    pos = torch.zeros(1, dtype=torch.int64, device=dev)
    scale = 1 / math.sqrt(D)
    outs = [None] * NL

    def two(with_attn=True):
        def f():
            for i in range(NL):
                q = kernels.int4_decode(x, ws[i][0], ws[i][1], g, norm_weight=nw, eps=1e-5,
                                        epilogue="rope_kv", rope=(freqs, pos, kcs[i], vcs[i], H))
                outs[i] = kernels.attn_decode(q, kcs[i], vcs[i], pos, scale) if with_attn else q
        return f

    def fused(S):
        def f():
            for i in range(NL):
                outs[i] = kernels.int4_qkv_attn(x, ws[i][0], ws[i][1], g, nw, 1e-5, freqs, pos,
                                                kcs[i], vcs[i], H, scale, S)
        return f

    for L in [int(v) for v in a.keys.split(",")]:
        pos.fill_(L - 1)
        ref = None
        for name, fn in (("two", two()), ("fused4", fused(4)), ("fused2", fused(2)),
                         ("fused1", fused(1)), ("gemv_only", two(False))):
            us = graph_us(fn, a.reps, NL, dev)
            rec = {"variant": name, "keys": L, "T": T, "us_per_layer_graph": round(us, 3)}
            if name != "gemv_only":
                fn()
                torch.cuda.synchronize()
                y = outs[0].float().reshape(-1)
                if ref is None:
                    ref = y
                else:
                    rec["rel_l2_vs_two"] = round(float((y - ref).norm() / ref.norm()), 6)
            print(json.dumps(rec), flush=True)
    kernels.check_decode_status()


if __name__ == "__main__":
    main()
