"""Prefill wqkv (Llama-3-8B: 6144x4096 int4 g32, M = 128 tokens) with and without the RoPE + KV
epilogue: us per launch in a HIP graph of 32 launches over distinct weights (as a prefill runs
the 32 layers), plain linear (tao_int4wo_linear_bf16 via torch.ops.torchao) vs the fused
tao_int4wo_linear_rope_kv_bf16. One JSON line per variant.

    PYTHONPATH=torchao-fork_amd python experiments/rope_epi_time.py
"""
import json
import math
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "torchao-fork_amd"))

from torchao._models.llama import kernels  # noqa: E402
from torchao._models.llama.model import ModelArgs, _rope_freqs  # noqa: E402


def graph_us(fn, n, dev, reps=20):
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
    dev = torch.device("cuda")
    H, Hkv, D, dim, g, NL, M, T = 32, 8, 128, 4096, 32, 32, 128, 328
    N = (H + 2 * Hkv) * D
    gen = torch.Generator(device=dev).manual_seed(0)
    ws = []
    for _ in range(NL):
        w = (torch.randn(N, dim, device=dev, generator=gen) / math.sqrt(dim)).to(torch.bfloat16)
        ws.append(torch.ops.torchao.int4_quantize_pack(w, g, 1e-6))
    x = torch.randn(1, M, dim, device=dev, dtype=torch.bfloat16, generator=gen)
    cfg = ModelArgs(n_layer=1, n_head=H, n_local_heads=Hkv, dim=dim, rope_base=500000)
    freqs = _rope_freqs(cfg, T).to(dev)
    pos = torch.arange(M, device=dev)
    kcs = [torch.zeros(1, Hkv, T, D, device=dev, dtype=torch.bfloat16) for _ in range(NL)]
    vcs = [torch.zeros(1, Hkv, T, D, device=dev, dtype=torch.bfloat16) for _ in range(NL)]

    def plain():
        for i in range(NL):
            torch.ops.torchao.int4_weight_only_linear(x.view(M, dim), ws[i][0], ws[i][1], g, None)

    def rope():
        for i in range(NL):
            kernels.int4_linear_rope_kv(x, ws[i][0], ws[i][1], g, freqs, pos, kcs[i], vcs[i], H)

    for name, fn in (("plain", plain), ("rope_kv", rope), ("plain", plain), ("rope_kv", rope)):
        print(json.dumps({"variant": name, "N": N, "K": dim, "M": M,
                          "us_per_launch_graph": round(graph_us(fn, NL, dev), 3)}), flush=True)


if __name__ == "__main__":
    main()
