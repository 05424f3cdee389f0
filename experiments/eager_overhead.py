"""Host cost per eager call of the quantized-linear ops at M = 1 (W8 of the round-1 verdict).

Launches each op back to back N times and reports wall µs per call after a synchronize: when
that exceeds the kernel time the op is host-bound and the number is its dispatch cost.

    python experiments/eager_overhead.py [N]
"""
import json
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, __file__.rsplit("/", 2)[0] + "/torchao-fork_amd")
import torchao  # noqa: E402,F401
from torchao.quantization import Int4WeightOnlyConfig, Int8WeightOnlyConfig, quantize_  # noqa: E402
from torchao.quantization import Int8DynamicActivationInt8WeightConfig  # noqa: E402


def per_call_us(fn, n):
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n * 1e6


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
    dev = "cuda"
    K = N = 4096
    x = torch.randn(1, K, device=dev, dtype=torch.bfloat16)
    res = {}
    res["empty_add_"] = per_call_us(lambda: x.add_(0), n)
    lin = torch.nn.Linear(K, N, bias=False, device=dev, dtype=torch.bfloat16)
    res["bf16_F.linear"] = per_call_us(lambda: F.linear(x, lin.weight), n)
    q4 = torch.nn.Sequential(torch.nn.Linear(K, N, bias=False, device=dev, dtype=torch.bfloat16))
    quantize_(q4, Int4WeightOnlyConfig(group_size=32))
    w = q4[0].weight
    impl = w.tensor_impl
    res["int4_op_direct"] = per_call_us(
        lambda: torch.ops.torchao.int4_weight_only_linear(x, impl.packed_weight,
                                                          impl.scale_and_zero, 32), n)
    res["int4_F.linear_aqt"] = per_call_us(lambda: F.linear(x, w), n)
    res["int4_module"] = per_call_us(lambda: q4(x), n)
    q8 = torch.nn.Sequential(torch.nn.Linear(K, N, bias=False, device=dev, dtype=torch.bfloat16))
    quantize_(q8, Int8WeightOnlyConfig())
    res["int8wo_module"] = per_call_us(lambda: q8(x), n)
    qd = torch.nn.Sequential(torch.nn.Linear(K, N, bias=False, device=dev, dtype=torch.bfloat16))
    quantize_(qd, Int8DynamicActivationInt8WeightConfig())
    res["int8dq_module"] = per_call_us(lambda: qd(x), n)
    # the reference's GPU op on its own tile format (PyTorch-ROCm aten)
    try:
        wt = torch.randint(0, 16, (N, K), dtype=torch.int32, device=dev)
        wu8 = (wt[:, ::2] << 4 | wt[:, 1::2]).to(torch.uint8)
        tile = torch.ops.aten._convert_weight_to_int4pack(wu8, 8)
        szr = torch.rand(K // 32, N, 2, device=dev, dtype=torch.bfloat16)
        res["aten_weight_int4pack_mm"] = per_call_us(
            lambda: torch.ops.aten._weight_int4pack_mm(x, tile, 32, szr), n)
    except Exception as e:  # build dependent
        res["aten_weight_int4pack_mm"] = f"{type(e).__name__}: {e}"[:200]
    print(json.dumps({k: (round(v, 2) if isinstance(v, float) else v) for k, v in res.items()}))


if __name__ == "__main__":
    main()
