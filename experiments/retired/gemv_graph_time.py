"""us per launch of the M = 1 int4 GEMV at the Llama-3-8B shapes, in a HIP graph of 32 launches
over 32 distinct weights (past the MALL), with the library TORCHAO_MI355X_LIB names (timing-only
variant builds: experiments/variant.sh gvN=int4_gemv:-DTAO_GEMV_DEBUG=N). One JSON line per shape.

    PYTHONPATH=torchao-fork_amd python experiments/gemv_graph_time.py
"""
import json
import os

import torch

from torchao import _lib

dev = torch.device("cuda")
lib = _lib.lib()
G = 32


def graph_us(launch, copies=32):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        launch()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            launch()
    torch.cuda.current_stream().wait_stream(s)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    v = []
    for _ in range(3):
        e0.record()
        for _ in range(10):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        v.append(e0.elapsed_time(e1) * 1e3 / 10 / copies)
    return sorted(v)[1]


def main():
    tag = os.path.basename(os.environ.get("TORCHAO_MI355X_LIB", "") or "shipped")
    tune = os.environ.get("TUNE")  # "rpw,wk,g,occ" -> tao_tune_int4_gemv (0 = built-in)
    if tune:
        _lib.call("tao_tune_int4_gemv", *[int(v) for v in tune.split(",")])
        tag += f" tune={tune}"
    shapes = os.environ.get("SHAPES", "4096x4096,6144x4096,28672x4096,4096x14336")
    for N, K in (tuple(int(v) for v in sh.split("x")) for sh in shapes.split(",")):
        ws = []
        for _ in range(32):
            q = torch.randint(0, 16, (N, K), dtype=torch.int32, device=dev)
            sz = (torch.rand(N, K // G, 2, device=dev) * 0.02).to(torch.bfloat16)
            ws.append((torch.ops.torchao.int4_pack(q), sz))
            del q
        x = torch.randn(1, K, device=dev, dtype=torch.bfloat16)
        y = torch.empty(N, device=dev, dtype=torch.bfloat16)

        def launch():
            sp = torch.cuda.current_stream().cuda_stream
            for p, z in ws:
                assert lib.tao_int4wo_linear_bf16(x.data_ptr(), p.data_ptr(), z.data_ptr(), None,
                                                  y.data_ptr(), 1, N, K, G, sp) == 0
        print(json.dumps({"lib": tag, "N": N, "K": K, "us_per_launch": round(graph_us(launch), 3)}),
              flush=True)
        del ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
