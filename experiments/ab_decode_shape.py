"""Interleaved A/B of launch shapes (tao_tune_int4_gemv rpw, wk, g, occ; 0,0,0,0 = built-in) of
the decode-fused int4 GEMV (RMSNorm prologue + RoPE/KV or SwiGLU epilogue, tao_int4wo_decode_bf16)
on one op of one model: graph of L launches over L weight copies (bench_decode.time_graph), the
configs alternated for R rounds; each config's output checked against the built-in's.

    python experiments/ab_decode_shape.py 70b wqkv_rope "0,0,0,0;4,2,1,8" 5
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import torch  # noqa: E402

from bench_decode import time_graph, weights  # noqa: E402
from torchao import _lib  # noqa: E402
from torchao._models.llama import kernels  # noqa: E402

DEV = "cuda"


def main():
    model, op = sys.argv[1], sys.argv[2]
    cfgs = [tuple(int(v) for v in c.split(",")) for c in sys.argv[3].split(";")]
    rounds = int(sys.argv[4]) if len(sys.argv) > 4 else 5
    L = 32
    K, H, Hkv, D, T, I = 4096, 32, 8, 128, 512, 14336
    if model == "70b":
        K, H, I = 8192, 64, 28672
    torch.manual_seed(0)
    x = torch.randn(1, 1, K, device=DEV, dtype=torch.bfloat16)
    nw = (torch.rand(K, device=DEV) + 0.5).to(torch.bfloat16)
    freqs = torch.randn(T, D // 2, 2, device=DEV)
    pos = torch.tensor([100], device=DEV)
    kc = torch.zeros(1, Hkv, T, D, device=DEV, dtype=torch.bfloat16)
    vc = torch.zeros_like(kc)
    N, epi = ((H + 2 * Hkv) * D, "rope_kv") if op == "wqkv_rope" else (2 * I, "swiglu")
    ws = weights(N, K, L)
    rope = (freqs, pos, kc, vc, H)

    def fused(i):
        p, sz, g = ws[i]
        return kernels.int4_decode(x, p, sz, g, norm_weight=nw, eps=1e-5, epilogue=epi, rope=rope)

    _lib.call("tao_tune_int4_gemv", 0, 0, 0, 0)
    ref = fused(0).float()
    res = {c: [] for c in cfgs}
    err = {}
    for _ in range(rounds):
        for c in cfgs:
            _lib.call("tao_tune_int4_gemv", *c)
            if c not in err:
                y = fused(0).float()
                err[c] = float((y - ref).norm() / ref.norm())
            res[c].append(round(time_graph(fused, L), 3))
    _lib.call("tao_tune_int4_gemv", 0, 0, 0, 0)
    for c, v in res.items():
        s = sorted(v)
        print(json.dumps({"model": model, "op": op, "rpw_wk_g_occ": list(c), "us": v,
                          "us_med": s[len(s) // 2], "rel_err_vs_builtin": err[c]}), flush=True)


if __name__ == "__main__":
    main()
