"""Decode-fused int4 GEMV (tao_int4wo_decode_bf16) vs the unfused chain it replaces, Llama-3-8B
shapes, one graph of L launches over L distinct weight copies (no cache reuse across layers,
like the real decode step). Prints one JSON line per (op, variant, tune shape).

    python experiments/bench_decode.py [--layers 32] [--sweep] [--model 8b|70b]
"""
import argparse
import itertools
import json

import torch

from torchao import _lib
from torchao._models.llama import kernels

DEV = "cuda"


def weights(N, K, L, g=32):
    ws = []
    for _ in range(L):
        packed = torch.randint(-2**31, 2**31 - 1, (N, K // 8), dtype=torch.int32, device=DEV)
        sz = (torch.rand(N, K // g, 2, device=DEV) * 0.01).to(torch.bfloat16)
        ws.append((packed, sz, g))
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
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", type=int, default=32)
    ap.add_argument("--sweep", action="store_true")
    ap.add_argument("--model", default="8b", choices=["8b", "70b"])
    args = ap.parse_args()
    L = args.layers
    K, H, Hkv, D, T, I = 4096, 32, 8, 128, 512, 14336
    if args.model == "70b":
        K, H, I = 8192, 64, 28672
    x = torch.randn(1, 1, K, device=DEV, dtype=torch.bfloat16)
    nw = (torch.rand(K, device=DEV) + 0.5).to(torch.bfloat16)
    freqs = torch.randn(T, D // 2, 2, device=DEV)
    pos = torch.tensor([100], device=DEV)
    kc = torch.zeros(1, Hkv, T, D, device=DEV, dtype=torch.bfloat16)
    vc = torch.zeros_like(kc)
    ops = {
        "wqkv_rope": (weights((H + 2 * Hkv) * D, K, L), "rope_kv"),
        "w13_swiglu": (weights(2 * I, K, L), "swiglu"),
        "head": (weights(128256, K, 2), "none"),
    }
    tunes = [(0, 0, 0, 0)]
    if args.sweep:
        tunes += [(r, w, g, o) for r, w, g, o in itertools.product((2, 4), (1, 2), (1, 2, 4, 8), (4, 8))
                  if w * g <= 8]
    for name, (ws, epi) in ops.items():
        n = len(ws)
        rope = (freqs, pos, kc, vc, H)

        def unfused(i):
            p, sz, g = ws[i]
            xn = kernels.rmsnorm(x, nw, 1e-5)
            y = torch.ops.torchao.int4_weight_only_linear(xn, p, sz, g)
            if epi == "swiglu":
                kernels.silu_mul(y)
            elif epi == "rope_kv":
                kernels.rope_kv(y, freqs, pos, kc, vc, H)

        def plain(i):
            p, sz, g = ws[i]
            torch.ops.torchao.int4_weight_only_linear(x, p, sz, g)

        for t in tunes:
            _lib.call("tao_tune_int4_gemv", *t)

            def fused(i, use_norm=True):
                p, sz, g = ws[i]
                kernels.int4_decode(x, p, sz, g, norm_weight=nw if use_norm else None, eps=1e-5,
                                    epilogue=epi, rope=rope)

            res = {"model": args.model, "op": name, "tune": t, "fused_us": round(time_graph(fused, n), 3),
                   "fused_nonorm_us": round(time_graph(lambda i: fused(i, False), n), 3)}
            # the prologue's LDS staging without the norm (tao_tune_int4_xlds 1): separates
            # the RMSNorm's own cost from staging x through LDS
            _lib.call("tao_tune_int4_xlds", 1)
            res["fused_lds_nonorm_us"] = round(time_graph(lambda i: fused(i, False), n), 3)
            _lib.call("tao_tune_int4_xlds", 0)
            _lib.call("tao_tune_int4_norm", 1)  # deferred RMSNorm scale
            res["fused_deferred_norm_us"] = round(time_graph(fused, n), 3)
            _lib.call("tao_tune_int4_norm", 0)
            if t == (0, 0, 0, 0):
                res["unfused_us"] = round(time_graph(unfused, n), 3)
                res["gemv_only_us"] = round(time_graph(plain, n), 3)
            print(json.dumps(res), flush=True)
        _lib.call("tao_tune_int4_gemv", 0, 0, 0, 0)


if __name__ == "__main__":
    main()
