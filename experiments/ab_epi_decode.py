"""Decode GEMVs whose epilogue reads operands (bias / residual, weight scale, RoPE position and
(cos, sin)): per-launch time in a HIP graph of L launches over distinct weights, plus an output
digest so two builds of the library (TORCHAO_MI355X_LIB) can be checked bit-identical.

    TORCHAO_MI355X_LIB=experiments/build/libold.so python experiments/ab_epi_decode.py TAG
"""
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "torchao-fork_amd"))
import torch  # noqa: E402

import torchao  # noqa: E402,F401
from torchao._models.llama import kernels  # noqa: E402
from bench_decode import time_graph, weights  # noqa: E402

DEV = "cuda"
L = 32


def digest(t):
    return hashlib.sha1(t.contiguous().view(torch.uint8).cpu().numpy().tobytes()).hexdigest()[:12]


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "run"
    torch.manual_seed(0)
    K, H, Hkv, D, T = 4096, 32, 8, 128, 512
    x1 = torch.randn(1, K, device=DEV, dtype=torch.bfloat16)
    x2 = torch.randn(1, 14336, device=DEV, dtype=torch.bfloat16)
    bias = torch.randn(4096, device=DEV, dtype=torch.bfloat16)
    nw = (torch.rand(K, device=DEV) + 0.5).to(torch.bfloat16)
    freqs = torch.randn(T, D // 2, 2, device=DEV)
    pos = torch.tensor([100], device=DEV)
    kc = torch.zeros(1, Hkv, T, D, device=DEV, dtype=torch.bfloat16)
    vc = torch.zeros_like(kc)
    w_o = weights(4096, 4096, L)
    w_2 = weights(4096, 14336, L)
    w_qkv = weights((H + 2 * Hkv) * D, K, L)
    w8 = [torch.randint(-127, 128, (4096, 4096), dtype=torch.int8, device=DEV) for _ in range(L)]
    s8 = (torch.rand(4096, device=DEV) * 0.01 + 1e-3).to(torch.bfloat16)

    def i4(ws, x, b):
        return lambda i: torch.ops.torchao.int4_weight_only_linear(x, ws[i][0], ws[i][1], 32, b)

    def qkv(i):
        p, sz, g = w_qkv[i]
        return kernels.int4_decode(x1, p, sz, g, norm_weight=nw, eps=1e-5, epilogue="rope_kv",
                                   rope=(freqs, pos, kc, vc, H))

    ops = {
        "int4_wo_bias": i4(w_o, x1, bias),
        "int4_w2_bias": i4(w_2, x2, bias),
        "int4_4096_nobias": i4(w_o, x1, None),
        "int4_wqkv_rope": qkv,
        "int8wo_bias": lambda i: torch.ops.torchao.int8_weight_only_linear(x1, w8[i], s8, bias),
        "int8wo_nobias": lambda i: torch.ops.torchao.int8_weight_only_linear(x1, w8[i], s8, None),
        "int8dyn_bias": lambda i: torch.ops.torchao.int8_dyn_linear(x1, w8[i], s8, bias),
    }
    rec = {"tag": tag}
    for name, fn in ops.items():
        out = fn(0)
        if name == "int4_wqkv_rope":  # q, and the cache rows written at pos
            out = torch.cat([out.flatten(), kc[:, :, 100].flatten(), vc[:, :, 100].flatten()])
        rec[name] = [round(time_graph(fn, L), 3), digest(out)]
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
