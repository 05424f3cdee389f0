"""Summarise a rocprofv3 kernel_trace.csv for the int4 GEMV: per (grid, block) shape, the
average duration of graph-replayed launches and of the last step's event-timed launches."""
import csv, sys, collections
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "int4wo_gemv" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
n_last = int(sys.argv[2]) if len(sys.argv) > 2 else 161
groups = {"replay": rows[:-n_last], "event_step": rows[-n_last:]}
for gname, rs in groups.items():
    agg = collections.defaultdict(list)
    for r in rs:
        key = (int(r["Grid_Size_X"]), int(r["Workgroup_Size_X"]))
        agg[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    tot = sum(sum(v) for v in agg.values())
    print(gname, "launches", len(rs), "total_us %.1f" % tot)
    for k, v in sorted(agg.items()):
        v.sort()
        print("   grid=%d block=%d n=%d avg_us=%.3f med_us=%.3f min_us=%.3f" % (k[0], k[1], len(v), sum(v)/len(v), v[len(v)//2], v[0]))
if groups["replay"]:
    first, last = groups["replay"][0], groups["replay"][-1]
    print("replay span_us %.1f" % ((int(last["End_Timestamp"]) - int(first["Start_Timestamp"])) / 1e3))
