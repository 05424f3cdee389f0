"""Interleaved A/B of int4 M=1 GEMV launch shapes (tao_tune_int4_gemv rpw, wk, g, occ) on one
weight shape: graph-replayed us per launch over rotated weights (sweep_gemv.graph_us), the
configs alternated for R rounds in one process; prints each config's values and median.

    python experiments/ab_gemv_shape.py 6144x4096 "2,2,4,0;2,1,4,0" 5
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "torchao-fork_amd"))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import torch  # noqa: E402

from sweep_gemv import bytes_of, graph_us  # noqa: E402
from torchao import _lib  # noqa: E402


def main():
    N, K = (int(v) for v in sys.argv[1].split("x"))
    cfgs = [tuple(int(v) for v in c.split(",")) for c in sys.argv[2].split(";")]
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    g = 32
    lib = _lib.lib()
    copies = max(4, min(64, int(400e6 // bytes_of(N, K))))
    ws = []
    for _ in range(copies):
        q = torch.randint(0, 16, (N, K), dtype=torch.int32, device="cuda")
        ws.append((torch.ops.torchao.int4_pack(q),
                   (torch.rand(N, K // g, 2, device="cuda") * 0.02).to(torch.bfloat16)))
        del q
    x = torch.randn(1, K, device="cuda", dtype=torch.bfloat16)
    ys = torch.empty(1, N, device="cuda", dtype=torch.bfloat16)
    reps = max(copies, 48)

    def run(n):
        st = torch.cuda.current_stream().cuda_stream
        for i in range(n):
            p, sz = ws[i % copies]
            lib.tao_int4wo_linear_bf16(x.data_ptr(), p.data_ptr(), sz.data_ptr(), None,
                                       ys.data_ptr(), 1, N, K, g, st)

    res = {c: [] for c in cfgs}
    for _ in range(rounds):
        for c in cfgs:
            _lib.call("tao_tune_int4_gemv", *c)
            res[c].append(round(graph_us(lambda: run(reps), reps), 3))
    _lib.call("tao_tune_int4_gemv", 0, 0, 0, 0)
    for c, v in res.items():
        s = sorted(v)
        print(json.dumps({"N": N, "K": K, "rpw_wk_g_occ": list(c), "us": v,
                          "us_med": s[len(s) // 2]}), flush=True)


if __name__ == "__main__":
    main()
