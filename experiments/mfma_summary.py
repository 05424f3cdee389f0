"""Summarise experiments/pmc_mfma.sh output: per config, the GEMM kernel's average duration
(kernel trace) and its MFMA busy fraction from the counters:
  util = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs * 1024 SIMDs)
(GRBM_GUI_ACTIVE is summed over the 8 XCDs, MI355X_MICROARCH.md 'DVFS give-back'; the busy
cycles are summed over every SIMD). python experiments/mfma_summary.py OUTDIR > summary.json"""

import csv
import glob
import json
import os
import statistics
import sys


def main():
    root = sys.argv[1]
    res = {}
    for d in sorted(glob.glob(os.path.join(root, "*/"))):
        tag = os.path.basename(d.rstrip("/"))
        kt = glob.glob(os.path.join(d, "kt", "**", "*kernel_trace.csv"), recursive=True)
        pm = glob.glob(os.path.join(d, "pmc", "**", "*counter_collection.csv"), recursive=True)
        if not kt or not pm:
            continue
        durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
                for r in csv.DictReader(open(kt[0])) if "gemm_mfma_kernel" in r["Kernel_Name"]]
        cnt = {}
        for r in csv.DictReader(open(pm[0])):
            if "gemm_mfma_kernel" not in r["Kernel_Name"]:
                continue
            cnt.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
        busy = statistics.median(cnt["SQ_VALU_MFMA_BUSY_CYCLES"])
        gui = statistics.median(cnt["GRBM_GUI_ACTIVE"])
        path, M, N, K = tag.split("_")
        M, N, K = int(M), int(N), int(K)
        us = statistics.median(durs)
        peak = 5000.0 if path == "int8dyn" else 2500.0
        res[tag] = {
            "launches": len(durs), "kernel_us_median": round(us, 2),
            "Tops_per_s": round(2 * M * N * K / (us * 1e-6) / 1e12, 1),
            "frac_of_dense_peak": round(2 * M * N * K / (us * 1e-6) / 1e12 / peak, 4),
            "SQ_VALU_MFMA_BUSY_CYCLES": busy, "GRBM_GUI_ACTIVE": gui,
            "mfma_busy_frac": round(busy / (gui / 8 * 1024), 4),
            "clock_GHz_est": round(gui / 8 / (us * 1e-6) / 1e9, 2),
        }
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
