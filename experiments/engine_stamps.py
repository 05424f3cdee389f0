"""Per-phase stamps of the decode FFN engine (tao_debug_ffn_engine_stamps): the last of L
chained layers in a replayed HIP graph; per workgroup the loader's and consumers' phase times
(us from the earliest loader entry of that launch), summarised as p50 / p90 / max over the 256
workgroups. python3 experiments/engine_stamps.py [--layers 8]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "torchao-fork_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from torchao import _lib  # noqa: E402
from torchao._models.llama import kernels  # noqa: E402

DIM, INTER, G = 4096, 14336, 32


def q(v):
    v = sorted(v)
    return [round(v[len(v) // 2], 3), round(v[int(len(v) * 0.9)], 3), round(v[-1], 3)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", type=int, default=8)
    ap.add_argument("--consumers", type=int, default=7)
    ap.add_argument("--dq", type=int, default=1)
    ap.add_argument("--ahead", type=int, default=3)
    ap.add_argument("--dyn", type=int, default=0)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    layers = []
    for i in range(args.layers):
        p13 = bench.make_int4_weight(2 * INTER, DIM, G, seed=10 * i + 1, device=dev)
        p2 = bench.make_int4_weight(DIM, INTER, G, seed=10 * i + 2, device=dev)
        layers.append((p13 + (G,), p2 + (G,), (torch.rand(DIM, device=dev) + 0.5).to(torch.bfloat16)))
    x0 = torch.randn(1, 1, DIM, device=dev, dtype=torch.bfloat16)
    st = torch.zeros(256 * 64, dtype=torch.int64, device=dev)
    lib = _lib.lib()
    assert lib.tao_tune_ffn_engine(args.consumers, args.dq, args.ahead, args.dyn) == 0

    def chain(x):
        for (p13, p2, nw) in layers:
            x = kernels.int4_ffn_engine(x, nw, 1e-5, p13, p2)
        return x

    chain(x0)
    torch.cuda.synchronize()
    assert lib.tao_debug_ffn_engine_stamps(st.data_ptr()) == 0
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=s):
            chain(x0)
    assert lib.tao_debug_ffn_engine_stamps(None) == 0
    torch.cuda.synchronize()
    out = {}
    for rep in range(3):
        st.zero_()
        graph.replay()
        torch.cuda.synchronize()
        t = st.view(256, 64).cpu().double()
        t0 = t[:, 0].min()
        us = lambda col: [(float(v) - float(t0)) / 100.0 for v in t[:, col]]  # noqa: E731
        dur = lambda col: [float(v) / 100.0 for v in t[:, col]]  # noqa: E731
        rec = {"loader_entry": q(us(0)), "loader_p1_issued": q(us(1)), "loader_all_issued": q(us(2)),
               "loader_last_full": q(us(3)), "loader_free_wait": q(dur(4))}
        for c in range(args.consumers):
            b = 8 + 6 * c
            rec[f"c{c}"] = {"norm": q(us(b)), "p1_done": q(us(b + 1)), "gather_done": q(us(b + 2)),
                            "p2_done": q(us(b + 3)), "end": q(us(b + 4)), "full_wait": q(dur(b + 5))}
        rec["end_max"] = round(max(max(us(8 + 6 * c + 4)) for c in range(args.consumers)), 3)
        # phase-1 completion of each workgroup (its last consumer) and its loader's phase-1 issue,
        # grouped by blockIdx % 8 (the XCD under round-robin placement)
        p1 = [max(us(8 + 6 * c + 1)[w] for c in range(args.consumers)) for w in range(256)]
        li = us(1)
        rec["by_wg_mod8"] = {str(x): {"p1_done": q([p1[w] for w in range(x, 256, 8)]),
                                      "loader_p1_issued": q([li[w] for w in range(x, 256, 8)])}
                             for x in range(8)}
        out[f"rep{rep}"] = rec
    print(json.dumps(out), flush=True)
    kernels.check_decode_status()


if __name__ == "__main__":
    main()
