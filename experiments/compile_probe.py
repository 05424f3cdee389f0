"""Does torch.compile(mode="reduce-overhead") put the int4 custom op inside its CUDA graph?
Prints per-call wall time of the compiled int4 two-linear model and the cudagraph skip log."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "torchao-fork_amd"))
import torch  # noqa: E402
import torch._inductor.config as icfg  # noqa: E402

from torchao.quantization import Int4WeightOnlyConfig, quantize_  # noqa: E402

torch._logging.set_logs(cudagraphs=True, perf_hints=True)
W = 4096
m = torch.nn.Sequential(torch.nn.Linear(W, W, bias=False), torch.nn.Linear(W, W, bias=False))
m = m.eval().to(torch.bfloat16).cuda()
quantize_(m, Int4WeightOnlyConfig(group_size=32))
x = torch.randn(1, W, dtype=torch.bfloat16, device="cuda")
with torch.no_grad():
    for name, fn in (("eager", m), ("compiled", torch.compile(m, mode="reduce-overhead"))):
        for _ in range(10):
            fn(x)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(200):
            fn(x)
        torch.cuda.synchronize()
        print(name, "us/call", round((time.perf_counter() - t0) / 200 * 1e6, 1), flush=True)
    prof = torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU,
                                              torch.profiler.ProfilerActivity.CUDA])
    cm = torch.compile(m, mode="reduce-overhead")
    for _ in range(5):
        cm(x)
    with prof:
        for _ in range(5):
            cm(x)
        torch.cuda.synchronize()
    print(prof.key_averages().table(sort_by="cpu_time_total", row_limit=15))
