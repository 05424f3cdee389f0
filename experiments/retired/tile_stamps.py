"""Per-workgroup phase timeline of gemm_tile_kernel from a TAO_TILE_STAMPS=1 build
(experiments/build/libtilestamps.so via TORCHAO_MI355X_LIB; experiments/tile_debug.sh builds it).
Stamps (s_memrealtime, 10 ns): 0 entry, 1 prologue done, 2 k loop done, 3 slab stored, 4
arrival/poll/claim done, 5 own part reduced, 6 last arriver's extra parts done; 7 = flags.
The last of 8 back-to-back launches leaves its stamps (steady state). Prints per configuration
the span, entry spread, per-phase median / max (µs), and how the parts were reduced.

    TORCHAO_MI355X_LIB=experiments/build/libtilestamps.so python experiments/tile_stamps.py
"""
import ctypes
import json

import numpy as np
import torch

from sweep_gemm import make_int4, make_int8dyn, make_int8wo
from torchao import _lib

lib = _lib.lib()
lib.tao_debug_tile_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
NB = 16384
CONFIGS = [("int8dyn", 128, 4096, 4096, 0), ("int8dyn", 128, 4096, 4096, 1),
           ("int4", 128, 4096, 4096, 0), ("int4", 128, 4096, 4096, 1),
           ("int4", 128, 28672, 4096, 0), ("int8wo", 128, 4096, 4096, 0)]


def stamps():
    buf = np.zeros(NB * 8, dtype=np.uint64)
    assert lib.tao_debug_tile_stamps(buf.ctypes.data, NB) == 0
    return buf.reshape(NB, 8)


def main():
    mk = {"int4": make_int4, "int8wo": make_int8wo, "int8dyn": make_int8dyn}
    for path, M, N, K, splits in CONFIGS:
        run, _ = mk[path](M, N, K)
        _lib.call("tao_tune_gemm_tile", 2, splits)
        for i in range(5):
            run(i)
        torch.cuda.synchronize()
        stamps()
        for i in range(8):
            run(i)
        torch.cuda.synchronize()
        s = stamps()
        idx = np.nonzero(s[:, 0] > 0)[0]
        s = s[idx].astype(np.int64)
        t0 = s[:, 0].min()
        us = lambda a: a / 100.0  # noqa: E731
        end = np.maximum(s[:, 5], s[:, 6])
        rec = {"path": path, "M": M, "N": N, "K": K, "splits": splits, "workgroups": int(len(s)),
               "span_us": round(float(us(end.max() - t0)), 2),
               "entry_spread_us": round(float(us(s[:, 0].max() - t0)), 2)}
        phases = [("prologue", 0, 1), ("k_loop", 1, 2)]
        if (s[:, 3] > 0).any():
            phases += [("slab_store", 2, 3), ("arrive_poll", 3, 4), ("own_part", 4, 5)]
        else:
            phases += [("epilogue", 2, 5)]
        for name, a, b in phases:
            d = us(s[:, b] - s[:, a])
            rec[name] = [round(float(np.median(d)), 2), round(float(d.max()), 2)]
        last = s[(s[:, 7] & 1) == 1]
        if len(last):
            d = us(last[:, 6] - last[:, 5])
            rec["last_extra_parts"] = [round(float(np.median(d)), 2), round(float(d.max()), 2)]
            rec["owners_claimed"] = int(((s[:, 7] & 2) == 2).sum())
        rec["loop_end_spread_us"] = round(float(us(s[:, 2].max() - s[:, 2].min())), 2)
        print(json.dumps(rec), flush=True)
    _lib.call("tao_tune_gemm_tile", 0, 0)


if __name__ == "__main__":
    main()
