"""Same-box A/B of the per-token int8 activation quantisation kernels (tao_tune_int8_quant):
0 = one wave per token with the token held in registers (default), 1 = one 256-thread block per
token. Kernel µs (dispatch-packet events), alternated twice per shape; outputs compared.

    python experiments/ab_quant.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "torchao-fork_amd"))
import torchao  # noqa: F401,E402
from torchao import _lib  # noqa: E402

SHAPES = [(128, 4096), (512, 4096), (2048, 4096), (128, 14336), (128, 8192), (32, 4096)]


def kernel_us(x, reps=50):
    torch.ops.torchao.int8_quantize_per_token(x)
    torch.cuda.synchronize()
    with _lib.KernelTimer(reps) as kt:
        for _ in range(reps):
            torch.ops.torchao.int8_quantize_per_token(x)
    torch.cuda.synchronize()
    d = sorted(kt.durations_ms)
    return d[len(d) // 2] * 1e3


def main():
    for M, K in SHAPES:
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16) * 3
        res = {"wave": [], "block": []}
        outs = {}
        for _ in range(2):
            for key, mode in (("wave", 0), ("block", 1)):
                _lib.call("tao_tune_int8_quant", mode)
                res[key].append(round(kernel_us(x), 2))
                outs[key] = torch.ops.torchao.int8_quantize_per_token(x)
        _lib.call("tao_tune_reset")
        same = all(torch.equal(a, b) for a, b in zip(outs["wave"], outs["block"]))
        print(json.dumps({"M": M, "K": K, "wave_us": res["wave"], "block_us": res["block"],
                          "identical": same}), flush=True)


if __name__ == "__main__":
    main()
