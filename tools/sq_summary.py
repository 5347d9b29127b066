"""Median per-launch SQ counters of one kernel from a rocprofv3 --pmc counter_collection.csv.
usage: python3 tools/sq_summary.py <csv> [kernel substring]"""
import collections
import csv
import statistics
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
pat = sys.argv[2] if len(sys.argv) > 2 else "closest4d"
by = collections.defaultdict(lambda: collections.defaultdict(float))
dur = {}
for r in rows:
    if pat not in r["Kernel_Name"]:
        continue
    by[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
    dur[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6
vals = collections.defaultdict(list)
for d, c in by.items():
    for k, v in c.items():
        vals[k].append(v)
out = {k: statistics.median(v) for k, v in sorted(vals.items())}
out["launch_ms_median"] = statistics.median(dur.values())
if "SQ_THREAD_CYCLES_VALU" in out and "SQ_ACTIVE_INST_VALU" in out:
    out["lane_utilisation"] = out["SQ_THREAD_CYCLES_VALU"] / (64 * out["SQ_ACTIVE_INST_VALU"])
print(out)
