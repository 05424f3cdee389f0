"""Persistent decode chain vs one launch per linear, Llama-3-8B (or 70B) linears, M = 1.

The chain: per layer wqkv (RMSNorm) -> wo (+ residual) -> w1||w3 (RMSNorm, SwiGLU) -> w2
(+ residual), 32 layers, then the head (RMSNorm): real data dependencies, one launch
(csrc/decode_chain.hip). Against the same linears as
  * fused: one tao_int4wo_decode_bf16 / int4 linear launch per linear (norm and SwiGLU fused,
    residual as bias), i.e. the e2e harness's launch sequence minus attention;
  * plain: the bench.py step (129 plain GEMV launches on independent inputs).
Each variant captured in one HIP graph, replayed back to back, HIP events on the replay stream.
Prints one JSON line per variant.

    python experiments/bench_chain.py [--model 8b|70b] [--layers N] [--reps R]
"""

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "torchao-fork_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from torchao._models.llama import kernels  # noqa: E402
from torchao.kernel.decode_chain import ChainPhase, DecodeChain  # noqa: E402


def build(cfg, n_layer, g, dev):
    D, I, V = cfg["dim"], cfg["intermediate"], cfg["vocab"]
    qkv = (cfg["n_head"] + 2 * cfg["n_kv_head"]) * cfg["head_dim"]
    gen = torch.Generator(device=dev).manual_seed(0)
    x0 = torch.randn(D, device=dev, dtype=torch.bfloat16, generator=gen)
    phases, layer_in, lp = [], x0, -1
    for li in range(n_layer):
        an = torch.empty(D, device=dev, dtype=torch.bfloat16).uniform_(0.5, 1.5, generator=gen)
        fn = torch.empty(D, device=dev, dtype=torch.bfloat16).uniform_(0.5, 1.5, generator=gen)
        ws = [bench.make_int4_weight(N, K, g, seed=100 * li + j, device=dev)
              for j, (N, K) in enumerate(((qkv, D), (D, D), (2 * I, D), (D, I)))]
        yq = torch.empty(qkv, device=dev, dtype=torch.bfloat16)
        h = torch.empty(D, device=dev, dtype=torch.bfloat16)
        gg = torch.empty(I, device=dev, dtype=torch.bfloat16)
        out = torch.empty(D, device=dev, dtype=torch.bfloat16)
        b = len(phases)
        phases += [
            ChainPhase(*ws[0], g, x=layer_in, y=yq, x_phase=lp, norm_w=an),
            ChainPhase(*ws[1], g, x=yq, y=h, x_phase=b, residual=layer_in),
            ChainPhase(*ws[2], g, x=h, y=gg, x_phase=b + 1, norm_w=fn, swiglu=True),
            ChainPhase(*ws[3], g, x=gg, y=out, x_phase=b + 2, residual=h),
        ]
        layer_in, lp = out, b + 3
    hn = torch.empty(D, device=dev, dtype=torch.bfloat16).uniform_(0.5, 1.5, generator=gen)
    head = bench.make_int4_weight(V, D, g, seed=7, device=dev)
    phases.append(ChainPhase(*head, g, x=layer_in, y=torch.empty(V, device=dev,
                                                                  dtype=torch.bfloat16),
                             x_phase=lp, norm_w=hn))
    return phases


def fused_step(phases):
    for p in phases:
        K = p.packed.shape[1] * 8
        x = p.x[:K].reshape(1, K)
        if p.swiglu or p.norm_w is not None:
            y = kernels.int4_decode(x, p.packed, p.scale_and_zero, p.group_size,
                                    norm_weight=p.norm_w, eps=p.eps,
                                    epilogue="swiglu" if p.swiglu else "none")
        else:
            y = torch.ops.torchao.int4_weight_only_linear(x, p.packed, p.scale_and_zero,
                                                          p.group_size, p.residual)
        p._out = y


def plain_step(phases, xs):
    for p in phases:
        K = p.packed.shape[1] * 8
        p._out = torch.ops.torchao.int4_weight_only_linear(xs[K], p.packed, p.scale_and_zero,
                                                           p.group_size, None)


def timed(fn, reps, dev):
    stream = torch.cuda.Stream(dev)
    stream.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(stream):
        fn()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=stream):
            fn()
        for _ in range(3):
            graph.replay()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(reps):
            graph.replay()
        e1.record(stream)
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="8b", choices=["8b", "70b"])
    ap.add_argument("--layers", type=int, default=0)
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--g", type=int, default=32)
    args = ap.parse_args()
    dev = torch.device("cuda")
    name, cfg = bench.MODELS[args.model]
    n_layer = args.layers or cfg["n_layer"]
    phases = build(cfg, n_layer, args.g, dev)
    nbytes = sum(bench.int4_alg_bytes(p.packed.shape[0], p.packed.shape[1] * 8, args.g)
                 for p in phases)
    chain = DecodeChain(phases)
    res = {}
    t0 = time.perf_counter()
    res["chain"] = timed(chain.run, args.reps, dev)
    chain.check()
    res["fused_launches"] = timed(lambda: fused_step(phases), args.reps, dev)
    xs = {K: torch.randn(1, K, device=dev, dtype=torch.bfloat16)
          for K in {p.packed.shape[1] * 8 for p in phases}}
    res["plain_launches"] = timed(lambda: plain_step(phases, xs), args.reps, dev)
    for k, ms in res.items():
        print(json.dumps({"variant": k, "model": name, "layers": n_layer, "phases": len(phases),
                          "ms_per_step": round(ms, 4),
                          "GBps": round(nbytes / (ms * 1e-3) / 1e9, 1),
                          "frac_of_8TBps": round(nbytes / (ms * 1e-3) / 8e12, 4),
                          "bytes_per_step": nbytes}), flush=True)
    print(json.dumps({"total_s": round(time.perf_counter() - t0, 1)}), flush=True)


if __name__ == "__main__":
    main()
