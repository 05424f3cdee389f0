"""Where the config-4 prefill (Llama-3-8B int4wo-32, 128-token prompt) spends its time: one eager
prefill after warm-up under torch.profiler, GPU kernel time summed per kernel name (top 25).

    PYTHONPATH=torchao-fork_amd python experiments/prefill_profile.py [--no_fuse_w13]
"""
import json

import torch

from torchao._models.llama.generate import apply_quantization, build_model, prefill


def main():
    import sys

    from torchao._models.llama import kernels

    if "--native" in sys.argv:
        kernels.PREFILL_ATTN = True
    dev = torch.device("cuda")
    model = build_model("Llama-3-8B", dev, seed=0)
    if "--no_fuse_w13" not in sys.argv:  # generate.py's default layout
        model.fuse_w13()
    apply_quantization(model, "int4wo-32")
    P, T = 128, 200
    model.setup_caches(1, P + T)
    model.enable_fused_kernels()
    prompt = torch.randint(0, model.config.vocab_size, (1, P), device=dev)
    pos = torch.arange(P, device=dev)
    for _ in range(3):
        prefill(model, prompt, pos)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    prefill(model, prompt, pos)
    e1.record()
    torch.cuda.synchronize()
    wall = e0.elapsed_time(e1)
    from torch.profiler import ProfilerActivity, profile

    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        prefill(model, prompt, pos)
        torch.cuda.synchronize()
    rows = []
    for ev in prof.key_averages():
        t = getattr(ev, "device_time_total", None) or getattr(ev, "cuda_time_total", 0)
        if t > 0:
            rows.append((t, ev.count, ev.key[:110]))
    rows.sort(reverse=True)
    print(json.dumps({"prefill_wall_ms_eager": round(wall, 3),
                      "gpu_us_total": round(sum(r[0] for r in rows), 1)}), flush=True)
    for t, n, k in rows[:25]:
        print(json.dumps({"us": round(t, 1), "calls": n, "kernel": k}), flush=True)


if __name__ == "__main__":
    main()
