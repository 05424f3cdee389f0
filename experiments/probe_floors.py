"""Kernel-duration floors on MI355X: empty launch, pure 16-B streaming reads of the int4 GEMV's
byte counts (weights rotated over > 256 MiB so the Infinity Cache cannot serve them), and the
int4 GEMV itself on the same sizes. Prints one JSON line per measurement."""

import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "torchao-fork_amd"))
import torch  # noqa: E402

lib = ctypes.CDLL(os.path.join(ROOT, "experiments", "libprobe.so"))
lib.probe_empty.restype = ctypes.c_float
lib.probe_empty.argtypes = [ctypes.c_int, ctypes.c_int]
lib.probe_read.restype = ctypes.c_float
lib.probe_read.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]


def med(xs):
    return statistics.median(xs)


def main():
    dev = torch.device("cuda")
    out = torch.zeros(1024, dtype=torch.int32, device=dev)
    for grid, block in [(1, 64), (256, 256), (256, 512), (1024, 256), (2048, 256), (4096, 512)]:
        ts = [lib.probe_empty(grid, block) for _ in range(50)]
        print(json.dumps({"probe": "empty", "grid": grid, "block": block, "us": round(med(ts) * 1e3, 3)}))

    for mb in [10.5, 15.75, 36.75, 328.6]:
        for block in (256, 512):
            for L in (1, 2, 4, 8, 16):
                unit = 16 * block * L
                bytes_ = int(mb * 1e6) // unit * unit
                copies = max(2, int(600e6 // bytes_))
                bufs = [torch.empty(bytes_, dtype=torch.uint8, device=dev) for _ in range(copies)]
                for b in bufs:
                    b.random_(0, 255)
                for nt in (0, 1):
                    ts = []
                    for r in range(3):
                        for b in bufs:
                            ts.append(lib.probe_read(b.data_ptr(), bytes_, block, L, nt, out.data_ptr()))
                    us = med(ts) * 1e3
                    print(json.dumps({"probe": "read", "MB": mb, "block": block, "L": L, "nt": nt,
                                      "us": round(us, 3), "GBps": round(bytes_ / us / 1e3, 1)}))
                del bufs
                torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
