"""Secondary measurements (BASELINE configs 2-3 and the prefill paths), one JSON line each.

* int8 dynamic activation x int8 weight, M = 128 (config 3): quant kernel + int8 MFMA GEMM,
  TOP/s against the MI355X int8 dense MFMA peak (2x bf16: ~5.0 POP/s) and weight GB/s; the
  incumbent torch._int_mm (hipBLASLt) + eager scaling beside it.
* int4 weight-only prefill, M in {8..512}: bf16-MFMA kernel TFLOP/s and GB/s; the incumbent
  dequantize -> torch.mm (hipBLASLt bf16) beside it.
* int8 weight-only decode, M = 1: GB/s.
Kernel durations from dispatch events (tao_profile_*), weights rotated past the 256 MiB MALL.
"""

import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "torchao-fork_amd"))
import torch  # noqa: E402

import torchao  # noqa: E402,F401
from torchao import _lib  # noqa: E402

BF16_PEAK = 2500.0  # TFLOP/s dense
I8_PEAK = 5000.0  # TOP/s dense


def med(xs):
    xs = sorted(xs)
    return xs[len(xs) // 2]


def timed_kernels(fn, launches_per_call, reps):
    fn()
    with _lib.KernelTimer(launches_per_call * reps) as kt:
        for i in range(reps):
            fn(i)
    d = kt.durations_ms
    per = [sum(d[i * launches_per_call:(i + 1) * launches_per_call]) for i in range(reps)]
    return med(per) * 1e3  # us


def wall_us(fn, reps=20):
    fn(0)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(reps):
        fn(i)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e6


def int8_dyn(M, N, K):
    copies = max(2, int(300e6 // (N * K)))
    ws = [torch.randint(-127, 128, (N, K), dtype=torch.int8, device="cuda") for _ in range(copies)]
    wsc = (torch.rand(N, device="cuda") * 0.01).to(torch.bfloat16)
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    qs = {}

    def run(i=0):
        q, s = torch.ops.torchao.int8_quantize_per_token(x)
        qs["q"], qs["s"] = q, s
        return torch.ops.torchao.int8_scaled_mm(q, s, ws[i % copies], wsc, None)

    us = timed_kernels(run, 2, 20)
    q, s = qs["q"], qs["s"]

    def gemm_only(i=0):
        return torch.ops.torchao.int8_scaled_mm(q, s, ws[i % copies], wsc, None)

    us_gemm = timed_kernels(gemm_only, 1, 20)

    def incumbent(i=0):
        c = torch._int_mm(q, ws[i % copies].t())
        return ((c.to(torch.bfloat16) * s) * wsc)

    us_inc = wall_us(incumbent)
    ops = 2 * M * N * K
    return {"path": "int8_dyn", "M": M, "N": N, "K": K, "us_quant+gemm": round(us, 2),
            "us_gemm": round(us_gemm, 2), "TOPs": round(ops / us_gemm / 1e6, 1),
            "mfma_frac": round(ops / us_gemm / 1e6 / I8_PEAK, 4),
            "weight_GBps": round(N * K / us_gemm / 1e3, 1),
            "incumbent_hipblaslt_wall_us": round(us_inc, 2)}


def int4_prefill(M, N, K, g=32):
    copies = max(2, int(300e6 // (N * K // 2)))
    ws = []
    for _ in range(copies):
        q = torch.randint(0, 16, (N, K), dtype=torch.int32, device="cuda")
        ws.append((torch.ops.torchao.int4_pack(q), (torch.rand(N, K // g, 2, device="cuda") * 0.02).to(torch.bfloat16)))
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)

    def run(i=0):
        p, sz = ws[i % copies]
        return torch.ops.torchao.int4_weight_only_linear(x, p, sz, g, None)

    us = timed_kernels(run, 1, 20)
    wdq = torch.ops.torchao.int4_dequantize(ws[0][0], ws[0][1], g, 0)

    def incumbent(i=0):
        return torch.mm(x, wdq.t())

    us_inc = wall_us(incumbent)
    flops = 2 * M * N * K
    byts = N * K // 2 + (K // g) * N * 4 + M * K * 2 + M * N * 2
    return {"path": "int4_prefill" if M > 4 else "int4_gemv", "M": M, "N": N, "K": K,
            "us": round(us, 2), "TFLOPs": round(flops / us / 1e6, 1),
            "mfma_frac": round(flops / us / 1e6 / BF16_PEAK, 4), "GBps": round(byts / us / 1e3, 1),
            "incumbent_bf16_mm_wall_us(dequantized W, L2/MALL warm)": round(us_inc, 2)}


def int8_wo(M, N, K):
    copies = max(2, int(300e6 // (N * K)))
    ws = [torch.randint(-127, 128, (N, K), dtype=torch.int8, device="cuda") for _ in range(copies)]
    s = (torch.rand(N, device="cuda") * 0.01).to(torch.bfloat16)
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)

    def run(i=0):
        return torch.ops.torchao.int8_weight_only_linear(x, ws[i % copies], s, None)

    us = timed_kernels(run, 1, 32)
    byts = N * K + 2 * N + 2 * M * K + 2 * M * N
    return {"path": "int8_wo", "M": M, "N": N, "K": K, "us": round(us, 2), "GBps": round(byts / us / 1e3, 1)}


def crossover_sweep():
    """int4 / int8-WO at M = 2..8 on both kernels (GEMV vs MFMA), 4096 x 4096 and 14336 x 4096."""
    for (N, K) in [(4096, 4096), (14336, 4096)]:
        for M in (2, 3, 4, 5, 6, 8):
            row = {"path": "crossover", "M": M, "N": N, "K": K}
            for mx, name in ((8, "gemv"), (1, "mfma")):
                _lib.call("tao_tune_linear_crossover", mx)
                row[f"int4_{name}_us"] = int4_prefill(M, N, K)["us"]
                row[f"int8wo_{name}_us"] = int8_wo(M, N, K)["us"]
            _lib.call("tao_tune_linear_crossover", 0)
            print(json.dumps(row), flush=True)


def main():
    if "--crossover" in sys.argv:
        crossover_sweep()
        return
    for (M, N, K) in [(128, 4096, 4096), (128, 14336, 4096), (128, 4096, 14336), (512, 4096, 4096)]:
        print(json.dumps(int8_dyn(M, N, K)), flush=True)
    for M in (5, 8, 16, 32, 64, 128, 256, 512):
        print(json.dumps(int4_prefill(M, 4096, 4096)), flush=True)
    print(json.dumps(int4_prefill(128, 14336, 4096)), flush=True)
    for (M, N, K) in [(1, 4096, 4096), (1, 14336, 4096), (1, 4096, 14336), (4, 4096, 4096), (16, 4096, 4096)]:
        print(json.dumps(int8_wo(M, N, K)), flush=True)


if __name__ == "__main__":
    main()
