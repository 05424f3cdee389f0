"""Sweep the MFMA skinny GEMM's launch shape (M tile x K splits) per path and shape.

One JSON line per (path, M, N, K): the auto choice's time and every forced (bm, splits) time,
kernel durations from dispatch events (tao_profile_*), weights rotated past the 256 MiB MALL.
Usage: python experiments/sweep_gemm.py [--quick]
"""

import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "torchao-fork_amd"))
import torch  # noqa: E402

import torchao  # noqa: E402,F401
from torchao import _lib  # noqa: E402


def med(xs):
    xs = sorted(xs)
    return xs[len(xs) // 2]


def kernel_us(fn, launches, reps=16):
    fn(0)
    torch.cuda.synchronize()
    with _lib.KernelTimer(launches * reps) as kt:
        for i in range(reps):
            fn(i)
    d = kt.durations_ms
    # the split-K GEMM is the last launch of each call
    return med([d[i * launches + launches - 1] for i in range(reps)]) * 1e3


def make_int4(M, N, K, g=32):
    copies = max(2, int(300e6 // (N * K // 2)))
    ws = []
    for _ in range(copies):
        q = torch.randint(0, 16, (N, K), dtype=torch.int32, device="cuda")
        sz = (torch.rand(N, K // g, 2, device="cuda") * 0.02).to(torch.bfloat16)
        ws.append((torch.ops.torchao.int4_pack(q), sz))
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)

    def run(i):
        p, sz = ws[i % copies]
        return torch.ops.torchao.int4_weight_only_linear(x, p, sz, g, None)

    return run, 1


def make_int8wo(M, N, K):
    copies = max(2, int(300e6 // (N * K)))
    ws = [torch.randint(-127, 128, (N, K), dtype=torch.int8, device="cuda") for _ in range(copies)]
    s = (torch.rand(N, device="cuda") * 0.01).to(torch.bfloat16)
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)

    def run(i):
        return torch.ops.torchao.int8_weight_only_linear(x, ws[i % copies], s, None)

    return run, 1


def make_int8dyn(M, N, K):
    copies = max(2, int(300e6 // (N * K)))
    ws = [torch.randint(-127, 128, (N, K), dtype=torch.int8, device="cuda") for _ in range(copies)]
    wsc = (torch.rand(N, device="cuda") * 0.01).to(torch.bfloat16)
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    q, s = torch.ops.torchao.int8_quantize_per_token(x)

    def run(i):
        return torch.ops.torchao.int8_scaled_mm(q, s, ws[i % copies], wsc, None)

    return run, 1


def weight_bytes(path, N, K, g=32):
    if path == "int4":
        return N * K // 2 + N * (K // g) * 4
    return N * K


def main():
    quick = "--quick" in sys.argv
    Ms = (8, 32, 128) if quick else (5, 8, 16, 32, 64, 128, 256, 512)
    shapes = [(4096, 4096), (14336, 4096), (4096, 14336)]
    makers = {"int4": make_int4, "int8wo": make_int8wo, "int8dyn": make_int8dyn}
    _lib.call("tao_tune_linear_crossover", 1)  # M >= 2 on the MFMA kernel
    for path, mk in makers.items():
        for (N, K) in shapes:
            for M in Ms:
                run, launches = mk(M, N, K)
                row = {"path": path, "M": M, "N": N, "K": K}
                _lib.call("tao_tune_gemm", 0, 0, 0)
                row["auto_us"] = round(kernel_us(run, launches), 2)
                best = (row["auto_us"], "auto")
                for bm in (16, 32, 64, 128):
                    if bm >= 4 * M and bm > 16:
                        continue
                    for kg in (1, 2, 4):
                        if kg * bm > 128:
                            continue
                        for sp in (1, 2, 4, 8):
                            _lib.call("tao_tune_gemm", bm, kg, sp)
                            us = round(kernel_us(run, launches), 2)
                            key = f"bm{bm}_kg{kg}_s{sp}"
                            row[key] = us
                            if us < best[0]:
                                best = (us, key)
                _lib.call("tao_tune_gemm", 0, 0, 0)
                row["best"] = best[1]
                row["best_us"] = best[0]
                row["best_weight_GBps"] = round(weight_bytes(path, N, K) / best[0] / 1e3, 1)
                row["best_TFLOPs"] = round(2 * M * N * K / best[0] / 1e6, 1)
                print(json.dumps(row), flush=True)
                del run
                torch.cuda.empty_cache()
    _lib.call("tao_tune_linear_crossover", 0)


if __name__ == "__main__":
    main()
