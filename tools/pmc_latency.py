"""Summarise tools/pmc_latency.sh: per-launch SQ counters of one kernel (median over its dispatches)
and the derived wave-time split.  usage: python3 tools/pmc_latency.py [gpurun_out/lat] [kernel]"""
import collections
import csv
import glob
import json
import statistics
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/lat"
kern = sys.argv[2] if len(sys.argv) > 2 else "k_trace_closest4d"
vals = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(f"{root}/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if kern not in r["Kernel_Name"]:
            continue
        vals[r["Counter_Name"]][(f, r["Dispatch_Id"])] += float(r["Counter_Value"])
c = {k: statistics.median(v.values()) for k, v in vals.items()}
out = {"kernel": kern, "counters": c}
W = c.get("SQ_WAVE_CYCLES")
if W:
    out["per_wave_cycle"] = {k: round(c[k] / W, 4) for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
                                                             "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_SCA",
                                                             "SQ_ACTIVE_INST_VMEM", "SQ_ACTIVE_INST_MISC") if k in c}
if c.get("SQ_INSTS_VMEM"):
    out["vmem_latency_cycles"] = round(c["SQ_INST_LEVEL_VMEM"] / c["SQ_INSTS_VMEM"], 1)
if c.get("SQ_INSTS_LDS"):
    out["lds_latency_cycles"] = round(c["SQ_INST_LEVEL_LDS"] / c["SQ_INSTS_LDS"], 1)
if c.get("SQ_INSTS_VALU") and c.get("SQ_THREAD_CYCLES_VALU"):
    out["valu_lane_util"] = round(c["SQ_THREAD_CYCLES_VALU"] / (64 * c.get("SQ_ACTIVE_INST_VALU", 1)), 4)
print(json.dumps(out, indent=1))
