"""Prefill attention per layer: tao_attn_prefill_bf16 (the MFMA flash kernel, attn_mfma.hip) against
the path it replaces, F.scaled_dot_product_attention over the caches with the causal mask
(gpt-fast Attention.forward at prefill), Llama-3-8B heads (32 q / 8 kv, D 128), B = 1, prompt
of S tokens at positions 0..S-1 in a cache of T rows. us per call from HIP events over 20 calls
after warm-up. One JSON line per S (time S >= 2048 before the kernel serves every
length).

    python experiments/attn_prefill_time.py [--S 128,512,2048,4096]
"""
import argparse
import json
import math
import os
import sys

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "torchao-fork_amd"))

from torchao._models.llama import kernels  # noqa: E402
from torchao.kernel.tuning import tuning  # noqa: E402


def graph_timed(fn, reps=20):
    """us per call from a HIP graph of `reps` calls (no host launch cost between them)."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(reps):
                fn()
    torch.cuda.current_stream().wait_stream(s)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(5):
        e0.record()
        g.replay()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3 / reps)
    return sorted(ts)[2]


def timed(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--S", default="128,512,2048,4096")
    a = ap.parse_args()
    dev = torch.device("cuda")
    H, Hkv, D = 32, 8, 128
    gen = torch.Generator(device=dev).manual_seed(0)
    for S in [int(v) for v in a.S.split(",")]:
        T = max(S, 1024)
        kc = torch.randn(1, Hkv, T, D, device=dev, dtype=torch.bfloat16, generator=gen)
        vc = torch.randn(1, Hkv, T, D, device=dev, dtype=torch.bfloat16, generator=gen)
        q = torch.randn(1, H, S, D, device=dev, dtype=torch.bfloat16, generator=gen)
        pos = torch.arange(S, device=dev)
        mask = torch.ones(T, T, dtype=torch.bool, device=dev).tril()[pos].view(1, 1, S, T)
        scale = 1.0 / math.sqrt(D)
        ours = timed(lambda: kernels.attn_prefill(q, kc, vc, pos, scale))
        by_nw = {}
        for nw in (1, 2, 4):  # waves per query block (key blocks split round-robin)
            with tuning(attn_prefill_nw=nw):
                by_nw[nw] = round(graph_timed(lambda: kernels.attn_prefill(q, kc, vc, pos,
                                                                            scale)), 2)
        sdpa = timed(lambda: F.scaled_dot_product_attention(q, kc, vc, attn_mask=mask,
                                                            enable_gqa=True))
        y = kernels.attn_prefill(q, kc, vc, pos, scale).float()
        r = F.scaled_dot_product_attention(q.float(), kc.float(), vc.float(), attn_mask=mask,
                                           enable_gqa=True).transpose(1, 2).reshape(1, S, H * D)
        err = float((y - r).abs().max())
        print(json.dumps({"lib": os.path.basename(os.environ.get("TORCHAO_MI355X_LIB", "shipped")),
                          "S": S, "T": T, "ours_us": round(ours, 2), "graph_us_by_nw": by_nw, "sdpa_us": round(sdpa, 2),
                          "speedup": round(sdpa / ours, 2), "max_abs_err_vs_fp32": round(err, 5)}),
              flush=True)
        del kc, vc, q, mask
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
