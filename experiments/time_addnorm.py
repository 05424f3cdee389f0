"""Kernel time of tao_add_rmsnorm_bf16 (dispatch-packet events, median of 50) per (rows, dim):
    [TORCHAO_MI355X_LIB=...] python experiments/time_addnorm.py >> out.jsonl
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "torchao-fork_amd"))
import torch  # noqa: E402

from torchao import _lib  # noqa: E402
from torchao._models.llama import kernels  # noqa: E402


def main():
    lib = os.path.basename(os.environ.get("TORCHAO_MI355X_LIB", "shipped"))
    g = torch.Generator(device="cuda").manual_seed(0)
    for rows, D in ((128, 4096), (1, 4096), (128, 8192), (512, 4096)):
        x = torch.randn(rows, D, device="cuda", generator=g).to(torch.bfloat16)
        r = torch.randn(rows, D, device="cuda", generator=g).to(torch.bfloat16)
        w = (torch.rand(D, device="cuda", generator=g) + 0.5).to(torch.bfloat16)
        kernels.add_rmsnorm(x, r, w, 1e-5)
        torch.cuda.synchronize()
        with _lib.KernelTimer(64) as kt:
            for _ in range(50):
                kernels.add_rmsnorm(x, r, w, 1e-5)
        torch.cuda.synchronize()
        d = sorted(kt.durations_ms)
        print(json.dumps({"lib": lib, "rows": rows, "dim": D, "us": round(d[len(d) // 2] * 1e3, 2),
                          "min_us": round(d[0] * 1e3, 2)}), flush=True)


if __name__ == "__main__":
    main()
