"""FETCH_SIZE of the int8 weight-only GEMV at M = 1 on bench.py's INT8WO_SHAPES.

run (on the GPU, under `rocprofv3 --pmc FETCH_SIZE`):
    python3 experiments/int8wo_pmc.py run
  launches each shape's GEMV L = 16 times eagerly over 16 distinct weight copies, shapes in
  INT8WO_SHAPES order (nothing else launches an int8 GEMV in between).
summarize (CPU):
    python3 experiments/int8wo_pmc.py summarize <counter_collection.csv> <out.json>
  takes the int8wo_gemv_kernel dispatches in dispatch order, L per shape, and writes
  hbm_bytes_per_launch per shape (FETCH_SIZE KiB x 1024 x 2, the gfx950 correction of
  MI355X_MICROARCH.md "HBM"); bench.py's int8wo_m1 block reads it (PMC_INT8WO_FILE).
"""
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
L = 16


def run():
    sys.path.insert(0, os.path.join(ROOT, "torchao-fork_amd"))
    import torch

    import bench
    from torchao import _lib

    lib = _lib.lib()
    dev = torch.device("cuda", 0)
    sp = torch.cuda.current_stream(dev).cuda_stream
    for (N, K) in bench.INT8WO_SHAPES:
        ws = [torch.randint(-127, 128, (N, K), dtype=torch.int8, device=dev) for _ in range(L)]
        sc = torch.full((N,), 1e-3, dtype=torch.bfloat16, device=dev)
        x = torch.randn(1, K, device=dev, dtype=torch.bfloat16)
        y = torch.empty(1, N, device=dev, dtype=torch.bfloat16)
        torch.cuda.synchronize()
        for c in range(L):
            assert lib.tao_int8wo_linear_bf16(x.data_ptr(), ws[c].data_ptr(), sc.data_ptr(), None,
                                              y.data_ptr(), 1, N, K, sp) == 0
        torch.cuda.synchronize()
        del ws
        torch.cuda.empty_cache()
    print("int8wo pmc run ok", flush=True)


def summarize(path, out):
    import bench

    rows = [r for r in csv.DictReader(open(path))
            if "int8wo_gemv_kernel" in r["Kernel_Name"] and r["Counter_Name"] == "FETCH_SIZE"]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    assert len(rows) == L * len(bench.INT8WO_SHAPES), len(rows)
    res = {"source": path, "counter": "FETCH_SIZE x 2 (gfx950 correction), bytes",
           "launches_per_shape": L, "hbm_bytes_per_launch": {}, "alg_bytes": {}}
    for i, (N, K) in enumerate(bench.INT8WO_SHAPES):
        vals = [float(r["Counter_Value"]) * 1024 * 2 for r in rows[i * L:(i + 1) * L]]
        res["hbm_bytes_per_launch"][f"{N}x{K}"] = round(sum(vals) / len(vals))
        res["alg_bytes"][f"{N}x{K}"] = bench.int8wo_alg_bytes(N, K)
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run()
    else:
        summarize(sys.argv[2], sys.argv[3])
