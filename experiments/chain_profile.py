"""Where the persistent decode chain's time goes: per-phase wall-clock stamps of every workgroup
(tao_chain_profile) for one run of the Llama-3-8B linears chain (experiments/bench_chain.py).

Per phase kind (wqkv / wo / w13 / w2 / head), medians over layers of:
  edge   = a workgroup's input-ready stamp minus the LAST producer's signal stamp (hand-off
           latency as the consumer sees it; median and max over workgroups)
  compute= tasks-done minus input-ready (the slowest workgroup: the phase's critical path)
  span   = last signal of the phase minus last signal of its input phase
Prints JSON lines."""

import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "torchao-fork_amd"))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "experiments"))

import torch  # noqa: E402

import bench  # noqa: E402
from bench_chain import build  # noqa: E402
from torchao.kernel.decode_chain import DecodeChain  # noqa: E402


def main():
    model = sys.argv[1] if len(sys.argv) > 1 else "8b"
    dev = torch.device("cuda")
    name, cfg = bench.MODELS[model]
    phases = build(cfg, cfg["n_layer"], 32, dev)
    chain = DecodeChain(phases)
    for _ in range(3):
        chain.run()
    prof = chain.profile(True)
    chain.run()
    torch.cuda.synchronize()
    chain.check()
    st = prof.cpu().double() / 100.0  # µs (100 MHz wall clock)
    kinds = ["wqkv", "wo", "w13", "w2"]
    per = {k: {"edge_med": [], "edge_max": [], "compute_max": [], "compute_med": [], "span": [],
               "sig_spread": []} for k in kinds + ["head"]}
    for p, ph in enumerate(phases):
        kind = "head" if p == len(phases) - 1 else kinds[p % 4]
        s = st[p]
        if ph.x_phase >= 0:
            prod_end = float(st[ph.x_phase, :, 3].max())
            edge = s[:, 1] - prod_end
            per[kind]["edge_med"].append(float(edge.median()))
            per[kind]["edge_max"].append(float(edge.max()))
            per[kind]["span"].append(float(s[:, 3].max()) - prod_end)
        comp = s[:, 2] - s[:, 1]
        per[kind]["compute_max"].append(float(comp.max()))
        per[kind]["compute_med"].append(float(comp.median()))
        per[kind]["sig_spread"].append(float(s[:, 3].max() - s[:, 3].min()))
    total = float(st[-1, :, 3].max() - st[0, :, 0].min())
    print(json.dumps({"model": name, "run_us": round(total, 1), "phases": len(phases)}))
    for k, d in per.items():
        print(json.dumps({"kind": k, **{m: round(statistics.median(v), 2) for m, v in d.items()
                                        if v}}))
    # the first two layers' phases, raw
    for p in range(8):
        s = st[p]
        print(json.dumps({"phase": p, "start_min": round(float(s[:, 0].min() - st[0, :, 0].min()), 2),
                          "ready_med": round(float(s[:, 1].median() - st[0, :, 0].min()), 2),
                          "done_max": round(float(s[:, 2].max() - st[0, :, 0].min()), 2),
                          "signal_max": round(float(s[:, 3].max() - st[0, :, 0].min()), 2)}))


if __name__ == "__main__":
    main()
