"""wo / w2 of a prefill in their partials form (tao_int4wo_linear_partials_f32, then
tao_add_rmsnorm_partials_bf16) under launch-shape overrides: per cfg (bn, wm, splits, stages,
a_steps, ks, loaders) the GEMM's and the norm's kernel us (dispatch-packet events, median) and
the pair's graph-replayed us over rotated weights, plus the rel. L2 of the norm input h against
the built-in route's (another split sums in another order).

    python experiments/time_partials.py 128x4096x14336 "64,2,4,4,0,0,0;64,2,8,4,0,0,0" [rounds]

With rounds > 1 the cfgs are timed in that many interleaved passes (same process) and each
record carries the per-pass values and their medians.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "torchao-fork_amd"))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import torch  # noqa: E402

from sweep_sf import median  # noqa: E402
from torchao import _lib  # noqa: E402
from torchao._models.llama import kernels  # noqa: E402

DEV = "cuda"


def main():
    M, N, K = (int(v) for v in sys.argv[1].split("x"))
    cfgs = [tuple(int(v) for v in c.split(",")) for c in sys.argv[2].split(";")]
    g = 32
    gen = torch.Generator(device=DEV).manual_seed(0)
    copies = max(2, int(320e6 // (N * K // 2)))
    w4 = []
    for _ in range(copies):
        q = torch.randint(0, 16, (N, K), dtype=torch.int32, device=DEV, generator=gen)
        sz = (torch.rand(N, K // g, 2, device=DEV, generator=gen) * 0.02).to(torch.bfloat16)
        w4.append((torch.ops.torchao.int4_pack(q), sz))
        del q
    x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16, generator=gen)
    res = torch.randn(M, N, device=DEV, dtype=torch.bfloat16, generator=gen)
    nw = (torch.rand(N, device=DEV, generator=gen) + 0.5).to(torch.bfloat16)
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    ref = None
    recs = {}
    for rnd in range(rounds):
        for ci, cfg in enumerate([None] + cfgs):
            _lib.call("tao_tune_reset")
            rec = recs.setdefault(ci, {"shape": sys.argv[1], "cfg": list(cfg) if cfg else "route",
                                       "gemm_us": [], "norm_us": [], "pair_graph_us": []})
            if "error" in rec:
                continue
            try:
                if cfg:
                    _lib.call("tao_tune_gemm_sf", 2, *cfg[:6])
                    _lib.call("tao_tune_gemm_sf_loaders", cfg[6])

                def pair(c):
                    part = kernels.int4_linear_partials(x, w4[c][0], w4[c][1], g)
                    if part is None:
                        raise RuntimeError("not served")
                    return part, kernels.add_rmsnorm_partials(res, part, nw, 1e-5)

                part, (h, _) = pair(0)
                torch.cuda.synchronize()
                rec["slices"] = int(part.shape[0])
                if ref is None:
                    ref = h.float()
                rec["rel_h"] = float(((h.float() - res.float()) - (ref - res.float())).norm()
                                     / (ref - res.float()).norm())
                for c in range(copies):
                    pair(c)
                torch.cuda.synchronize()
                reps = 30
                with _lib.KernelTimer(reps * 2 + 4) as kt:
                    for i in range(reps):
                        pair(i % copies)
                torch.cuda.synchronize()
                d = kt.durations_ms
                rec["gemm_us"].append(round(median(d[0::2]) * 1e3, 2))
                rec["norm_us"].append(round(median(d[1::2]) * 1e3, 2))
                # graph: copies x (partials, norm) back to back, replayed
                s = torch.cuda.Stream()
                s.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(s):
                    pair(0)
                    graph = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(graph, stream=s):
                        for c in range(copies):
                            pair(c)
                torch.cuda.current_stream().wait_stream(s)
                for _ in range(3):
                    graph.replay()
                torch.cuda.synchronize()
                ts = []
                for _ in range(10):
                    e0 = torch.cuda.Event(enable_timing=True)
                    e1 = torch.cuda.Event(enable_timing=True)
                    e0.record()
                    graph.replay()
                    e1.record()
                    torch.cuda.synchronize()
                    ts.append(e0.elapsed_time(e1) / copies)
                rec["pair_graph_us"].append(round(median(ts) * 1e3, 2))
                del graph
            except RuntimeError as e:
                rec["error"] = str(e)[:160]
    for rec in recs.values():
        for k in ("gemm_us", "norm_us", "pair_graph_us"):
            if rec[k]:
                rec[k + "_med"] = median(rec[k])
        print(json.dumps(rec), flush=True)
    _lib.call("tao_tune_reset")


if __name__ == "__main__":
    main()
