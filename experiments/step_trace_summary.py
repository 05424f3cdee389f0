"""Per-step kernel time of bench.py's decode step from a rocprofv3 kernel_trace.csv.

python3 experiments/step_trace_summary.py <kernel_trace.csv> <bench line .json> <out.json>

Finds every window of consecutive int4 GEMV launches whose (grid, block) sequence is the step's
(the first window fixes the pattern: 129 launches = 32 x {wqkv, wo, w1||w3, w2} + head), i.e. the
replays of the whole-step graph, and reports per step: the sum of the kernels' durations, the
span (first start -> last end), and per shape the average duration; beside them the paired bench
line's ms_per_step / kernel_ms_per_step / roofline.frac and the frac recomputed from the profile
(alg bytes per step / per-step kernel-duration sum, and / per-step span).
"""
import csv
import json
import sys


def main():
    path, line_path, out = sys.argv[1:4]
    line = None
    for ln in open(line_path):
        ln = ln.strip()
        if ln.startswith("{"):
            line = json.loads(ln)
    n = line["roofline"]["launches"]
    alg = line["roofline"]["alg_bytes_per_step"]
    rows = [r for r in csv.DictReader(open(path)) if "int4wo_gemv" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    key = [(int(r["Grid_Size_X"]), int(r["Workgroup_Size_X"])) for r in rows]
    # the step's pattern: its per-layer 4-shape cycle x 32 + head (first window with distinct
    # neighbours at the layer stride)
    pat = None
    for i in range(len(rows) - n + 1):
        w = key[i:i + n]
        if len(set(w)) >= 4 and all(w[j] == w[j + 4] for j in range(n - 5)) and w[-1] != w[-5]:
            pat = w
            break
    assert pat is not None, "no whole-step window in the trace"
    steps, i = [], 0
    while i <= len(rows) - n:
        if key[i:i + n] == pat:
            rs = rows[i:i + n]
            d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rs]
            span = (int(rs[-1]["End_Timestamp"]) - int(rs[0]["Start_Timestamp"])) / 1e3
            steps.append((sum(d), span, d))
            i += n
        else:
            i += 1
    shapes = {}
    for _, _, d in steps:
        for k, v in zip(pat, d):
            shapes.setdefault(k, []).append(v)
    ksum = sum(s[0] for s in steps) / len(steps)
    span = sum(s[1] for s in steps) / len(steps)
    res = {"trace": path, "bench_line": line_path, "steps_found": len(steps),
           "launches_per_step": n,
           "kernel_sum_us_per_step": round(ksum, 2), "span_us_per_step": round(span, 2),
           "per_shape_avg_us": {f"grid{k[0]}xblock{k[1]}": round(sum(v) / len(v), 3)
                                for k, v in shapes.items()},
           "line_ms_per_step": line["ms_per_step"],
           "line_kernel_ms_per_step": line["roofline"]["kernel_ms_per_step"],
           "line_frac": line["roofline"]["frac"],
           "frac_from_kernel_sum": round(alg / (ksum * 1e-6) / 1e9 / 8000.0, 4),
           "frac_from_span": round(alg / (span * 1e-6) / 1e9 / 8000.0, 4),
           "kernel_sum_le_ms_per_step": ksum * 1e-3 <= line["ms_per_step"]}
    res["frac_rel_diff_span"] = round(res["frac_from_span"] / res["line_frac"] - 1, 4)
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
