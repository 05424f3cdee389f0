"""Summarise a rocprofv3 --pmc FETCH_SIZE pass of bench.py into per-shape HBM traffic.

python experiments/pmc_summary.py <counter_collection.csv> <out.json> [launches_per_step=161]

FETCH_SIZE on gfx950 counts half the bytes of a wide coalesced streaming read
(MI355X_MICROARCH.md "HBM": TCC_EA0_RDREQ x 64 B for 128-B requests), so the summary doubles it.
Kernels are grouped by (grid, workgroup) size, i.e. by GEMV shape.
"""

import collections
import csv
import json
import sys


def main():
    path, out = sys.argv[1], sys.argv[2]
    per_step = int(sys.argv[3]) if len(sys.argv) > 3 else 161
    rows = list(csv.DictReader(open(path)))
    per_kernel = collections.defaultdict(list)
    for r in rows:
        if "int4wo_gemv_kernel" not in r["Kernel_Name"] or r["Counter_Name"] != "FETCH_SIZE":
            continue
        key = (int(r["Grid_Size"]), int(r["Workgroup_Size"]))
        per_kernel[key].append(float(r["Counter_Value"]) * 1024 * 2)  # KiB -> B, x2 gfx950
    summary = {"source": path, "counter": "FETCH_SIZE x 2 (gfx950 correction), bytes",
               "per_grid": {}}
    total, launches = 0.0, 0
    for (grid, wg), vals in sorted(per_kernel.items()):
        avg = sum(vals) / len(vals)
        summary["per_grid"][f"{grid}x{wg}"] = {"launches": len(vals), "hbm_bytes_avg": round(avg)}
        total += sum(vals)
        launches += len(vals)
    summary["launches"] = launches
    summary["hbm_bytes_per_launch_avg"] = round(total / max(launches, 1))
    summary["hbm_bytes_total"] = round(total)
    summary["launches_per_step"] = per_step
    summary["steps"] = launches / per_step
    summary["hbm_bytes_per_step"] = round(total / (launches / per_step))
    json.dump(summary, open(out, "w"), indent=1)
    print(json.dumps(summary))


if __name__ == "__main__":
    main()
