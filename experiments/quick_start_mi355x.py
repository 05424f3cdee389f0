"""The reference's quick-start flow (scripts/quick_start.py: a two-linear toy model,
quantize_(Int4WeightOnlyConfig(group_size=32)), torch.compile, benchmark_model) run on this
package unchanged at the API level, plus the same model eager and at Llama-sized widths.
Prints one JSON line per configuration: bf16 and int4 mean ms per forward and the speedup."""

import copy
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "torchao-fork_amd"))
import torch  # noqa: E402

from torchao.quantization import Int4WeightOnlyConfig, quantize_  # noqa: E402
from torchao.utils import benchmark_model  # noqa: E402


class TwoLinear(torch.nn.Module):
    def __init__(self, d_in: int, d_hidden: int, d_out: int):
        super().__init__()
        self.linear1 = torch.nn.Linear(d_in, d_hidden, bias=False)
        self.linear2 = torch.nn.Linear(d_hidden, d_out, bias=False)

    def forward(self, x):
        return self.linear2(self.linear1(x))


@torch.no_grad()
def run(width: int, compile_mode, num_runs: int = 100):
    torch.manual_seed(0)
    base = TwoLinear(width, width, width).eval().to(torch.bfloat16).to("cuda")
    q = copy.deepcopy(base)
    quantize_(q, Int4WeightOnlyConfig(group_size=32))
    x = torch.randn(1, width, dtype=torch.bfloat16, device="cuda")
    ref = base(x)
    err = float((q(x).float() - ref.float()).norm() / ref.float().norm())
    if compile_mode is not None:
        torch._dynamo.reset()
        base = torch.compile(base, mode=compile_mode, fullgraph=True)
        q = torch.compile(q, mode=compile_mode, fullgraph=True)
    for m in (base, q):  # compile / autotune / graph capture outside the timed runs
        for _ in range(5):
            m(x)
    t_bf16 = benchmark_model(base, num_runs, (x,))
    t_int4 = benchmark_model(q, num_runs, (x,))
    return {"width": width, "compile": compile_mode, "bf16_ms": round(t_bf16, 4),
            "int4_ms": round(t_int4, 4), "speedup": round(t_bf16 / t_int4, 2),
            "int4_vs_bf16_rel_l2": round(err, 4)}


def main():
    for width in (1024, 4096, 8192):
        for mode in (None, "max-autotune", "reduce-overhead"):
            try:
                rec = run(width, mode)
            except Exception as e:  # report, keep going
                rec = {"width": width, "compile": mode, "error": f"{type(e).__name__}: {e}"[:400]}
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
