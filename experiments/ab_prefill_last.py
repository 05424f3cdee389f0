"""Same-process A/B of a prefill flag of torchao/_models/llama/kernels.py (default
PREFILL_LAST_ROW: the greedy prefill's last block on the one-token kernels; PREFILL_PARTIALS: wo /
w2's K slices summed by the following add + RMSNorm) at BASELINE config 4 (Llama-3-8B int4wo-32,
fused w1||w3, 128-token prompt): two prefill graphs captured with the flag off / on, replayed
alternately; ms per replay (HIP events around each replay), median of each, and the first tokens
of both.

    PYTHONPATH=torchao-fork_amd python experiments/ab_prefill_last.py [FLAG | tune:KNOB=OFF,ON]
"""
import contextlib
import json
import sys

import torch

from torchao._models.llama import kernels
from torchao._models.llama.generate import GraphPrefill, apply_quantization, build_model
from torchao.kernel.tuning import tuning


def main():
    dev = torch.device("cuda")
    model = build_model("Llama-3-8B", dev, seed=0)
    model.fuse_w13()
    apply_quantization(model, "int4wo-32")
    P = 128
    model.setup_caches(1, P + 200)
    model.enable_fused_kernels()
    gen = torch.Generator(device="cpu").manual_seed(1)
    name = sys.argv[1] if len(sys.argv) > 1 else "PREFILL_LAST_ROW"
    pres = {}
    for flag in (False, True):
        if name.startswith("tune:"):  # tune:KNOB=OFF,ON -- the knob's values for off / on
            knob, vals = name[5:].split("=")
            ctx = tuning(**{knob: int(vals.split(",")[int(flag)])})
        else:
            setattr(kernels, name, flag)
            ctx = contextlib.nullcontext()
        with ctx:
            pres[flag] = GraphPrefill(model, (1, P), dev)
            pres[flag].capture(torch.randint(0, model.config.vocab_size, (1, P),
                                             generator=gen).to(dev))
    if not name.startswith("tune:"):
        setattr(kernels, name, True)
    times = {False: [], True: []}
    toks = {False: [], True: []}
    for rep in range(8):
        prompt = torch.randint(0, model.config.vocab_size, (1, P), generator=gen).to(dev)
        for flag in ((False, True) if rep % 2 == 0 else (True, False)):
            for _ in range(3):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                tok = pres[flag](prompt)
                e1.record()
                e1.synchronize()
                times[flag].append(e0.elapsed_time(e1))
            toks[flag].append(int(tok.item()))
    for flag in (False, True):
        v = sorted(times[flag])
        print(json.dumps({"flag": name, "on": flag, "ms_median": round(v[len(v) // 2], 4),
                          "ms_min": round(v[0], 4), "n": len(v)}), flush=True)
    print(json.dumps({"first_tokens_equal": toks[False] == toks[True], "off": toks[False],
                      "on": toks[True]}), flush=True)


if __name__ == "__main__":
    main()
