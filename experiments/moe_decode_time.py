"""MoE decode FFN per layer, Mixtral-8x7B shapes (E = 8 experts, top-2, dim 4096, intermediate
14336, int4 g32), one token: the reference's one-token branch (index the 3-D weights by the top-k
experts, then per-expert F.linear on the AQT; _models/mixtral-moe/model.py:360-384) against
kernels.int4_moe_ffn_decode (three grouped launches). L layers of distinct weights in one HIP
graph, us per layer; outputs compared bit for bit.

    PYTHONPATH=torchao-fork_amd python experiments/moe_decode_time.py
"""
import json
import math
import os
import sys

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "torchao-fork_amd"))

from torchao._models.llama import kernels  # noqa: E402
from torchao.dtypes import TensorCoreTiledLayout, to_affine_quantized_intx  # noqa: E402
from torchao.quantization.quant_primitives import MappingType, ZeroPointDomain  # noqa: E402

DEV = "cuda"


def quant3d(E, N, K, seed):
    g = torch.Generator(device=DEV).manual_seed(seed)
    w = ((torch.rand(E, N, K, device=DEV, generator=g) * 2 - 1) / math.sqrt(K)).to(torch.bfloat16)
    return to_affine_quantized_intx(
        w, MappingType.ASYMMETRIC, (1, 1, 32), torch.int32, 0, 15, 1e-6,
        zero_point_dtype=torch.bfloat16, preserve_zero=False,
        zero_point_domain=ZeroPointDomain.FLOAT, _layout=TensorCoreTiledLayout(8))


def reference_branch(x, w1, w2, w3, ei, ew):
    A = ei.numel()
    idx = ei.view(A)
    w1s, w2s, w3s = w1[idx], w2[idx], w3[idx]
    outs = []
    for i in range(A):
        y1 = F.silu(F.linear(x, w1s[i]))
        y3 = F.linear(x, w3s[i])
        outs.append(F.linear(y1 * y3, w2s[i]))
    return (torch.cat(outs, dim=0) * ew.view(-1, 1)).sum(dim=0).unsqueeze(-1)


def graph_us(fn, n, reps=10):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(3):
        e0.record()
        for _ in range(reps):
            g.replay()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3 / reps / n)
    return sorted(ts)[1]


def main():
    E, A, D, I, L = 8, 2, 4096, 14336, 4
    layers = [(quant3d(E, I, D, 3 * i), quant3d(E, D, I, 3 * i + 1), quant3d(E, I, D, 3 * i + 2))
              for i in range(L)]
    gen = torch.Generator(device=DEV).manual_seed(9)
    x = torch.randn(1, D, device=DEV, dtype=torch.bfloat16, generator=gen)
    ew, ei = torch.topk(F.softmax(torch.randn(1, E, device=DEV, generator=gen), -1), A, -1)
    ew = (ew / ew.sum(-1, keepdim=True)).to(torch.bfloat16)
    outs = {}

    def ref():
        outs["ref"] = [reference_branch(x, w1, w2, w3, ei, ew) for w1, w2, w3 in layers]

    def grouped():
        outs["grouped"] = [kernels.int4_moe_ffn_decode(x, w1, w2, w3, ei, ew)
                           for w1, w2, w3 in layers]

    bytes_per_layer = 3 * A * D * I // 2 + 3 * A * D * (I // 32) * 4
    for name, fn in (("reference_branch", ref), ("grouped", grouped),
                     ("reference_branch", ref), ("grouped", grouped)):
        us = graph_us(fn, L)
        print(json.dumps({"variant": name, "E": E, "top_k": A, "dim": D, "inter": I,
                          "us_per_layer_graph": round(us, 2),
                          "GBps_active_experts": round(bytes_per_layer / us / 1e3, 1)}), flush=True)
    ref()
    grouped()
    torch.cuda.synchronize()
    print(json.dumps({"bit_identical": all(torch.equal(a, b) for a, b in
                                           zip(outs["ref"], outs["grouped"]))}), flush=True)


if __name__ == "__main__":
    main()
