"""Attribution of the prefill tile family's LDS-DMA intake (tao_sf_intake_probe modes) at the int4
M = 128 4096^2 route: 0 the tile's pieces (bench.py's intake_probe), 1 weight + (scale, zero)
pieces only, 2 x pieces only, 3 every piece with x from a private copy per workgroup, 4 / 5 the
tile's / x pieces with each workgroup's k steps rotated; plus the
GEMM itself and mode 0 at 3 stages. Kernel us (dispatch events, median), 3 interleaved rounds.

    python experiments/intake_modes.py
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


def main():
    M, N, K, g = 128, 4096, 4096, 32
    gen = torch.Generator(device=DEV).manual_seed(0)
    copies = max(2, int(320e6 // (N * K // 2)))
    w4 = []
    for _ in range(copies):
        q = torch.randint(0, 16, (N, K), dtype=torch.int32, device=DEV, generator=gen)
        sz = (torch.rand(N, K // g, 2, device=DEV, generator=gen) * 0.02).to(torch.bfloat16)
        w4.append((torch.ops.torchao.int4_pack(q), sz))
        del q
    x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16, generator=gen)
    xp = torch.randn(256 * 128, K, device=DEV, dtype=torch.bfloat16, generator=gen)
    sink = torch.zeros(1024, dtype=torch.int32, device=DEV)
    shp = (ctypes.c_int * 7)()
    h = _lib.lib()

    def probe(mode):
        xx = xp if mode == 3 else x

        def run(c):
            rc = h.tao_sf_intake_probe(0, mode, xx.data_ptr(), w4[c][0].data_ptr(),
                                       w4[c][1].data_ptr(), M, N, K, g,
                                       ctypes.cast(shp, ctypes.c_void_p), sink.data_ptr(),
                                       torch.cuda.current_stream().cuda_stream)
            if rc != 0:
                raise RuntimeError(h.tao_last_error().decode())
        return run

    def gemm(c):
        torch.ops.torchao.int4_weight_only_linear(x, w4[c][0], w4[c][1], g, None)

    def timed(fn, reps=30):
        for c in range(copies):
            fn(c)
        torch.cuda.synchronize()
        with _lib.KernelTimer(reps + 4) as kt:
            for i in range(reps):
                fn(i % copies)
        torch.cuda.synchronize()
        return median(kt.durations_ms) * 1e3

    cases = [("gemm", None, gemm), ("probe_tile", None, probe(0)), ("probe_w_z_only", None, probe(1)),
             ("probe_x_only", None, probe(2)), ("probe_x_private", None, probe(3)),
             ("probe_tile_rotated", None, probe(4)), ("probe_x_only_rotated", None, probe(5)),
             ("probe_tile_3stages", (64, 2, 4, 3), probe(0)), ("gemm_3stages", (64, 2, 4, 3), gemm),
             ("probe_tile_8issuers", (64, 2, 4, 4, "off"), probe(0)),
             ("probe_x_only_8issuers", (64, 2, 4, 4, "off"), probe(2)),
             ("gemm_no_loaders", (64, 2, 4, 4, "off"), gemm),
             ("probe_tile_8loaders", (64, 2, 4, 4, "8"), probe(0)),
             ("probe_x_only_8loaders", (64, 2, 4, 4, "8"), probe(2)),
             ("gemm_8loaders", (64, 2, 4, 4, "8"), gemm),
             ("gemm_8loaders_3stages", (64, 2, 4, 3, "8"), gemm)]
    _lib.call("tao_tune_reset")
    y0 = torch.ops.torchao.int4_weight_only_linear(x, w4[0][0], w4[0][1], g, None)
    _lib.call("tao_tune_gemm_sf", 2, 64, 2, 4, 4, 0, 0)
    _lib.call("tao_tune_gemm_sf_loaders", 3)
    y1 = torch.ops.torchao.int4_weight_only_linear(x, w4[0][0], w4[0][1], g, None)
    print(json.dumps({"gemm_8loaders_bit_identical_to_route": bool(torch.equal(y0, y1))}),
          flush=True)
    res = {c[0]: [] for c in cases}
    for _ in range(3):
        for name, cfg, fn in cases:
            _lib.call("tao_tune_reset")
            if cfg:
                _lib.call("tao_tune_gemm_sf", 2, *cfg[:4], 0, 0)
                _lib.call("tao_tune_gemm_sf_loaders",
                          {("off",): 1, ("8",): 3}.get(tuple(cfg[4:]), 2))
            res[name].append(round(timed(fn), 2))
    _lib.call("tao_tune_reset")
    for name, v in res.items():
        print(json.dumps({"case": name, "us": v, "us_med": sorted(v)[1]}), flush=True)


if __name__ == "__main__":
    main()
