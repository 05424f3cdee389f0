"""Per-token kernel budget of an e2e decode run from a rocprofv3 kernel trace CSV
(rocpd2csv output): kernels grouped by (short name, grid, block), count / avg / total us,
normalised per decoded token (argv[2] = decoded tokens in the trace)."""
import collections
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
tokens = float(sys.argv[2])
agg = collections.defaultdict(list)
for r in rows:
    name = r["Kernel_Name"]
    m = re.search(r"(\w+_kernel)(<[^(]*>)?", name)
    short = (m.group(1) + (m.group(2) or "")) if m else name[:60]
    key = (short[:90], int(r["Grid_Size_X"]) * int(r.get("Grid_Size_Y", 1) or 1),
           int(r["Workgroup_Size_X"]))
    agg[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
tot = 0.0
out = []
for k, v in agg.items():
    per_tok = len(v) / tokens
    if per_tok < 0.5:
        continue
    out.append((sum(v) / tokens, per_tok, sum(v) / len(v), k))
for t, n, a, k in sorted(out, reverse=True):
    tot += t
    print("%8.1f us/tok  %6.1f launches/tok  avg %7.2f us  %s grid=%d blk=%d" % (t, n, a, k[0], k[1], k[2]))
print("total %.1f us/token, %.1f launches/token" % (tot, sum(o[1] for o in out)))
