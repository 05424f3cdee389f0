"""Per-workgroup phase timeline of gemm_mfma_kernel from a TAO_GEMM_STAMPS=1 build
(experiments/build/libstamps.so via TORCHAO_MI355X_LIB): one launch after warm-up; stamps
(s_memrealtime, 10 ns) at entry, prologue done, k loop done, k-group reduction done, end.
Prints per configuration: kernel span, dispatch spread of the entries, and medians / maxima of
each phase (us).

    TORCHAO_MI355X_LIB=experiments/build/libstamps.so python experiments/gemm_stamps.py [--b2b]

--b2b: stamps of the last of 8 back-to-back launches (steady state) instead of one launch on an
idle GPU.
"""
import ctypes
import json
import statistics

import numpy as np
import torch

from sweep_gemm import make_int4, make_int8dyn
from torchao import _lib

lib = _lib.lib()
lib.tao_debug_gemm_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
NB = 16384
BACK_TO_BACK = False


def stamps():
    buf = np.zeros(NB * 8, dtype=np.uint64)
    rc = lib.tao_debug_gemm_stamps(buf.ctypes.data, NB)
    assert rc == 0
    return buf.reshape(NB, 8)


def run_one(tag, run, shape):
    _lib.call("tao_tune_gemm", *shape)
    for i in range(5):
        run(i)
    torch.cuda.synchronize()
    stamps()  # clear
    if BACK_TO_BACK:  # steady state: the last of 8 queued launches leaves its stamps
        for i in range(8):
            run(i)
    else:
        run(0)
    torch.cuda.synchronize()
    s = stamps()
    idx = np.nonzero(s[:, 0] > 0)[0]
    s = s[idx].astype(np.int64)
    t0 = s[:, 0].min()
    us = lambda a: (a / 100.0)  # noqa: E731  (100 MHz)
    e0 = s[:, 6].min()
    rec = {"config": tag, "shape": shape, "workgroups": int(len(s)),
           "span_us": round(float(us(s[:, 4].max() - e0)), 2),
           "first_instr_spread_us": round(float(us(s[:, 6].max() - e0)), 2),
           "setup": [round(float(np.median(us(s[:, 0] - s[:, 6]))), 2),
                     round(float(us(s[:, 0] - s[:, 6]).max()), 2)],
           "entry_spread_us": round(float(us(s[:, 0].max() - t0)), 2)}
    for name, a, b in (("prologue", 0, 1), ("k_loop", 1, 2), ("kgroup_red", 2, 3), ("tail", 3, 4)):
        d = us(s[:, b] - s[:, a])
        rec[name] = [round(float(np.median(d)), 2), round(float(d.max()), 2)]
    last = s[s[:, 5] == 1]
    if len(last):
        rec["last_arriver_tail"] = [round(float(np.median(us(last[:, 4] - last[:, 3]))), 2),
                                    round(float(us(last[:, 4] - last[:, 3]).max()), 2)]
    # per XCD (blocks b, b + 8, ... share one): first-instruction offset of its earliest and
    # latest block relative to the grid's first
    per = []
    for x in range(8):
        sel = s[idx % 8 == x, 6]
        if len(sel):
            per.append([round(float(us(sel.min() - e0)), 2), round(float(us(sel.max() - e0)), 2)])
    rec["per_xcd_first_last_us"] = per
    order = np.argsort(idx)
    rec["first_instr_by_block_us_first16"] = [round(float(us(s[order[i], 6] - e0)), 2)
                                             for i in range(min(16, len(order)))]
    # how many workgroups were resident at once: entries before the first exit
    first_exit = s[:, 4].min()
    rec["entered_before_first_exit"] = int((s[:, 0] < first_exit).sum())
    print(json.dumps(rec), flush=True)


def main():
    global BACK_TO_BACK
    import sys
    BACK_TO_BACK = "--b2b" in sys.argv
    _lib.call("tao_tune_linear_crossover", 1)
    _lib.call("tao_tune_gemm_algo", 1)
    _lib.call("tao_tune_gemm_table", 1)
    run, _ = make_int8dyn(128, 4096, 4096)
    run_one("int8dyn 128x4096x4096", run, (32, 2, 1))
    run_one("int8dyn 128x4096x4096", run, (32, 1, 1))
    run, _ = make_int4(128, 4096, 4096)
    run_one("int4 128x4096x4096", run, (64, 1, 4))
    run_one("int4 128x4096x4096", run, (32, 2, 1))
    run, _ = make_int4(128, 28672, 4096)
    run_one("int4 128x28672x4096", run, (64, 2, 1))
    _lib.call("tao_tune_gemm", 0, 0, 0)


if __name__ == "__main__":
    main()
