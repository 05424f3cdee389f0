"""Per-workgroup phase timeline of the single-fetch GEMM (csrc/gemm_sf.hip) from a TAO_SF_STAMPS=1
build (experiments/build/libsfst.so, loaded through TORCHAO_MI355X_LIB): s_memrealtime stamps
(100 MHz) of every workgroup of the last of 40 back-to-back launches. Per phase: median / max over
workgroups of the time since the first workgroup's entry (us).

    TORCHAO_MI355X_LIB=experiments/build/libsfst.so python experiments/sf_stamps.py
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "torchao-fork_amd"))
import torch  # noqa: E402

import torchao  # noqa: E402,F401
from torchao import _lib  # noqa: E402

DEV = "cuda"
NAMES = ["entry", "issued", "landed0", "loop_done", "seam_done", "end"]


def stamps(n):
    buf = (ctypes.c_ulonglong * (n * 8))()
    fn = _lib.lib().tao_debug_sf_stamps
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
    assert fn(ctypes.cast(buf, ctypes.c_void_p), n) == 0
    return [list(buf[i * 8:(i + 1) * 8]) for i in range(n)]


def pct(v, q):
    v = sorted(v)
    return v[min(len(v) - 1, int(q * len(v)))] if v else None


def run_case(path, M, N, K, cfg, gen, out, seam=1):
    if path == "int8":
        copies = max(2, int(320e6 // (N * K)))
        ws = [torch.randint(-127, 128, (N, K), dtype=torch.int8, device=DEV, generator=gen)
              for _ in range(copies)]
        wsc = (torch.rand(N, device=DEV, generator=gen) * 0.01 + 1e-3).to(torch.bfloat16)
        x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16, generator=gen)
        xq, xs = torch.ops.torchao.int8_quantize_per_token(x)
        fn = lambda c: torch.ops.torchao.int8_scaled_mm(xq, xs, ws[c], wsc, None)  # noqa: E731
    else:
        copies = max(2, int(320e6 // (N * K // 2)))
        w4 = []
        for _ in range(copies):
            q = torch.randint(0, 16, (N, K), dtype=torch.int32, device=DEV, generator=gen)
            sz = (torch.rand(N, K // 32, 2, device=DEV, generator=gen) * 0.02).to(torch.bfloat16)
            w4.append((torch.ops.torchao.int4_pack(q), sz))
        x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16, generator=gen)
        fn = lambda c: torch.ops.torchao.int4_weight_only_linear(x, w4[c][0], w4[c][1], 32, None)  # noqa: E731
    _lib.call("tao_tune_gemm_sf", 2, *cfg)
    _lib.call("tao_tune_gemm_sf_seam", seam)
    for i in range(40):
        fn(i % copies)
    torch.cuda.synchronize()
    bn, splits = cfg[0], cfg[2]
    ntiles = (N + bn - 1) // bn
    nwg = ntiles * splits * ((M + 127) // 128)
    st = stamps(nwg)
    t0 = min(r[0] for r in st)
    rec = {"path": path, "M": M, "N": N, "K": K, "cfg": list(cfg), "seam": seam, "wgs": nwg}
    for k, name in enumerate(NAMES):
        vals = [(r[k] - t0) / 100.0 for r in st if r[k]]
        rec[name] = ([round(pct(vals, 0.0), 2), round(pct(vals, 0.5), 2), round(pct(vals, 1.0), 2)]
                     if vals else None)
    red = [r for r in st if r[7] >= 1]  # the fixed reducer, or every spread-seam workgroup
    pub = [r for r in st if r[7] == 0]
    rec["reducer_loop_us"] = round(pct([(r[3] - r[2]) / 100 for r in red], 0.5), 2)
    rec["reducer_wait_us"] = (round(pct([(r[4] - r[3]) / 100 for r in red], 0.5), 2)
                              if splits > 1 and red else 0)
    rec["reducer_epi_us"] = (round(pct([(r[5] - r[4]) / 100 for r in red], 0.5), 2)
                             if splits > 1 and red else 0)
    if pub:
        rec["pub_loop_us"] = round(pct([(r[3] - r[2]) / 100 for r in pub], 0.5), 2)
        rec["pub_end_med"] = round(pct([(r[5] - t0) / 100 for r in pub], 0.5), 2)
    rec["first_land_us"] = round(pct([(r[2] - r[0]) / 100 for r in st], 0.5), 2)
    print(json.dumps(rec), flush=True)
    out.write(json.dumps(rec) + "\n")
    _lib.call("tao_tune_reset")


def main():
    out = open(os.path.join(ROOT, "gpurun_out", "r4_sf_stamps.jsonl"), "a")
    gen = torch.Generator(device=DEV).manual_seed(0)
    for cfg in [(32, 8, 2, 3, 0, 256), (64, 4, 4, 3, 0, 128), (128, 4, 8, 2, 0, 256),
                (64, 4, 8, 3, 0, 128)]:
        run_case("int8", 128, 4096, 4096, cfg, gen, out)
    for cfg in [(64, 2, 4, 3, 0, 0), (64, 2, 2, 3, 0, 0), (128, 2, 8, 2, 0, 0), (64, 2, 4, 2, 0, 0)]:
        run_case("int4", 128, 4096, 4096, cfg, gen, out)


if __name__ == "__main__":
    main()
