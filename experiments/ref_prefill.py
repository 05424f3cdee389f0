"""The reference's own GPU path for the M = 128 prefill linears, timed on this box beside ours
(VERDICT r3 "Missing 3"): config 3 as safe_int_mm -> torch._int_mm (hipBLASLt int8) + the
int_scaled_matmul epilogue (kernel/intmm.py:82,136-142; plain_layout.py:301-315), and int4 g32 at
M = 128 as aten._weight_int4pack_mm (tensor_core_tiled_layout.py:104). Each op's calls captured
in one HIP graph over weight copies rotated past the MALL; us per call from events on the replay
stream (launch gaps included, the same for both sides)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "torchao-fork_amd"))
import torch  # noqa: E402

import torchao  # noqa: E402,F401

DEV = "cuda"


def graph_us(fn, copies, reps=3):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for c in range(copies):
            fn(c)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for c in range(copies):
                fn(c)
        g.replay()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(reps):
            g.replay()
        e1.record(s)
    e1.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps / copies


def main(M=128, N=4096, K=4096, g=32):
    gen = torch.Generator(device=DEV).manual_seed(0)
    res = {"M": M, "N": N, "K": K}
    copies = max(2, int(320e6 // (N * K)))
    ws = [torch.randint(-127, 128, (N, K), dtype=torch.int8, device=DEV, generator=gen)
          for _ in range(copies)]
    wsc = (torch.rand(N, device=DEV, generator=gen) * 0.01 + 1e-3).to(torch.bfloat16)
    x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16, generator=gen)
    xq, xs = torch.ops.torchao.int8_quantize_per_token(x)
    xs2 = xs.reshape(-1, 1)

    def ref8(c):  # safe_int_mm + int_scaled_matmul + w scale (the reference's GPU ops)
        cc = torch._int_mm(xq, ws[c].t())
        y = (cc * xs2).to(torch.bfloat16)
        return y * wsc

    def ours8(c):
        return torch.ops.torchao.int8_scaled_mm(xq, xs, ws[c], wsc, None)
    res["int8_ref_graph_us"] = round(graph_us(ref8, copies), 2)
    res["int8_ours_graph_us"] = round(graph_us(ours8, copies), 2)
    res["int8_ref_intmm_only_us"] = round(graph_us(lambda c: torch._int_mm(xq, ws[c].t()), copies), 2)
    a, b = ref8(0).float(), ours8(0).float()
    res["int8_rel_l2"] = float((a - b).norm() / b.norm())
    del ws
    copies = max(2, int(320e6 // (N * K // 2)))
    w4, wr = [], []
    for _ in range(copies):
        q = torch.randint(0, 16, (N, K), dtype=torch.int32, device=DEV, generator=gen)
        sz = (torch.rand(N, K // g, 2, device=DEV, generator=gen) * 0.02).to(torch.bfloat16)
        w4.append((torch.ops.torchao.int4_pack(q), sz))
        u8 = ((q[:, ::2] << 4) | q[:, 1::2]).to(torch.uint8)
        wr.append((torch.ops.aten._convert_weight_to_int4pack(u8, 8), sz.transpose(0, 1).contiguous()))
        del q, u8
    res["int4_ref_graph_us"] = round(graph_us(
        lambda c: torch.ops.aten._weight_int4pack_mm(x, wr[c][0], g, wr[c][1]), copies), 2)
    res["int4_ours_graph_us"] = round(graph_us(
        lambda c: torch.ops.torchao.int4_weight_only_linear(x, w4[c][0], w4[c][1], g, None), copies), 2)
    a = torch.ops.aten._weight_int4pack_mm(x, wr[0][0], g, wr[0][1]).float()
    b = torch.ops.torchao.int4_weight_only_linear(x, w4[0][0], w4[0][1], g, None).float()
    res["int4_rel_l2"] = float((a - b).norm() / b.norm())
    print(json.dumps(res), flush=True)
    with open(os.path.join(ROOT, "gpurun_out", "r4_ref_prefill.jsonl"), "a") as f:
        f.write(json.dumps(res) + "\n")


if __name__ == "__main__":
    main()
