"""What a prefill GEMM launch pays once: dispatch-event us of (a) a near-empty
launch (tao_hbm_read_probe over 8 KiB: one workgroup), (b) the read probe over 1 MiB (256
workgroups), (c) the LDS-DMA intake probe of the 4096-column route shape at K = 512 ... 4096
(1 .. 8 k steps per slice, no compute), (d) the GEMM itself at the same K.

    python experiments/fixed_cost_probe.py
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "torchao-fork_amd"))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import torch  # noqa: E402

from sweep_sf import median  # noqa: E402
from torchao import _lib  # noqa: E402

DEV = "cuda"


def timed(fn, copies, reps=40):
    for c in range(copies):
        fn(c)
    torch.cuda.synchronize()
    with _lib.KernelTimer(reps + 4) as kt:
        for i in range(reps):
            fn(i % copies)
    torch.cuda.synchronize()
    return round(median(kt.durations_ms) * 1e3, 2)


def main():
    h = _lib.lib()
    sink = torch.zeros(1024, dtype=torch.int32, device=DEV)
    st = lambda: torch.cuda.current_stream().cuda_stream  # noqa: E731
    buf = torch.zeros(1 << 20, dtype=torch.uint8, device=DEV)
    out = {}
    out["read_probe_8KiB_us"] = timed(lambda c: h.tao_hbm_read_probe(buf.data_ptr(), 8192, sink.data_ptr(), st()), 1)
    out["read_probe_1MiB_us"] = timed(lambda c: h.tao_hbm_read_probe(buf.data_ptr(), 1 << 20, sink.data_ptr(), st()), 1)
    M, N, g = 128, 4096, 32
    gen = torch.Generator(device=DEV).manual_seed(0)
    shp = (ctypes.c_int * 7)()
    for K in (512, 1024, 2048, 4096):
        copies = max(2, int(320e6 // (N * K // 2)))
        w4 = []
        for _ in range(copies):
            q = torch.randint(0, 16, (N, K), dtype=torch.int32, device=DEV, generator=gen)
            sz = (torch.rand(N, K // g, 2, device=DEV, generator=gen) * 0.02).to(torch.bfloat16)
            w4.append((torch.ops.torchao.int4_pack(q), sz))
            del q
        x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16, generator=gen)
        _lib.call("tao_tune_gemm_sf", 2, 64, 2, 4, 4, 0, 0)
        _lib.call("tao_tune_gemm_sf_loaders", 2)

        def probe(c):
            rc = h.tao_sf_intake_probe(0, 0, x.data_ptr(), w4[c][0].data_ptr(), w4[c][1].data_ptr(),
                                       M, N, K, g, ctypes.cast(shp, ctypes.c_void_p),
                                       sink.data_ptr(), st())
            if rc != 0:
                raise RuntimeError(h.tao_last_error().decode())

        def gemm(c):
            torch.ops.torchao.int4_weight_only_linear(x, w4[c][0], w4[c][1], g, None)

        out[f"K{K}"] = {"steps_per_slice": K // 128 // 4, "intake_probe_us": timed(probe, copies),
                        "gemm_us": timed(gemm, copies)}
        _lib.call("tao_tune_reset")
        del w4
        torch.cuda.empty_cache()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
