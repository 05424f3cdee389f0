"""Summarise experiments/pmc_prefill.sh's counter passes (one JSON line per GEMM configuration).

python experiments/pmc_prefill_summary.py gpurun_out/r2_pmc_prefill > profiles/r2_pmc_prefill.jsonl

Per configuration, medians over the GEMM dispatches (kernel names containing "gemm": gemm_mfma_kernel, gemm32_int4_kernel, ...) of every
counter, plus derived ratios:
  wait_frac        = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES (both quad-cycles: the share of wave
                     time spent waiting on an instruction dependency, mostly vmcnt / lgkmcnt)
  lds_conflict_frac= SQ_LDS_BANK_CONFLICT / SQ_ACTIVE_INST_LDS (extra cycles per LDS cycle)
  mfma_busy_frac   = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE x CUs)
  hbm_bytes        = FETCH_SIZE x 1024 x 2 (KiB; gfx950 counts half of a 128-B streaming read,
                     MI355X_MICROARCH.md), against the algorithmic bytes of the GEMM
"""

import collections
import csv
import glob
import json
import os
import re
import statistics
import sys

CUS = 256


def alg_bytes(path, M, N, K, g=32):
    if path == "int8dyn":
        return N * K + N * 2 + M * K + M * 2 + M * N * 2
    return N * K // 2 + (K // g) * N * 4 + M * K * 2 + M * N * 2


def main():
    root = sys.argv[1]
    for cfg in sorted(os.listdir(root)):
        d = os.path.join(root, cfg)
        if not os.path.isdir(d):
            continue
        path, M, N, K = cfg.split("_")
        M, N, K = int(M), int(N), int(K)
        path = "int8dyn" if path.startswith("sfint8") else "int4" if path.startswith("sfint4") else path
        vals = collections.defaultdict(list)
        for f in glob.glob(os.path.join(d, "p*", "*_counter_collection.csv")):
            for r in csv.DictReader(open(f)):
                if "gemm" not in r["Kernel_Name"]:
                    continue
                vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
        med = {k: statistics.median(v) for k, v in vals.items()}
        us = None
        log = os.path.join(d, "p1.log")
        if os.path.exists(log):
            m = re.search(r": ([0-9.]+) us", open(log).read())
            us = float(m.group(1)) if m else None
        rec = {"config": cfg, "kernel_us": us, "counters": {k: round(v, 1) for k, v in med.items()}}
        g = lambda k: med.get(k)  # noqa: E731
        if g("SQ_WAIT_INST_ANY") and g("SQ_WAVE_CYCLES"):
            rec["wait_frac"] = round(g("SQ_WAIT_INST_ANY") / g("SQ_WAVE_CYCLES"), 3)
        if g("SQ_LDS_BANK_CONFLICT") is not None and g("SQ_ACTIVE_INST_LDS"):
            rec["lds_conflict_frac"] = round(g("SQ_LDS_BANK_CONFLICT") / g("SQ_ACTIVE_INST_LDS"), 3)
        if g("SQ_VALU_MFMA_BUSY_CYCLES") and g("GRBM_GUI_ACTIVE"):
            rec["mfma_busy_frac"] = round(g("SQ_VALU_MFMA_BUSY_CYCLES")
                                          / (g("GRBM_GUI_ACTIVE") * CUS), 4)
        if g("FETCH_SIZE"):
            hb = g("FETCH_SIZE") * 1024 * 2
            rec["hbm_bytes"] = int(hb)
            rec["alg_bytes"] = alg_bytes(path, M, N, K)
            rec["hbm_over_alg"] = round(hb / rec["alg_bytes"], 3)
        if g("SQ_INSTS_LDS") and g("SQ_INSTS_MFMA"):
            rec["lds_insts_per_mfma"] = round(g("SQ_INSTS_LDS") / g("SQ_INSTS_MFMA"), 2)
        if g("SQ_INSTS_VALU") and g("SQ_INSTS_MFMA"):
            rec["valu_insts_per_mfma"] = round(g("SQ_INSTS_VALU") / g("SQ_INSTS_MFMA"), 2)
        print(json.dumps(rec))


if __name__ == "__main__":
    main()
