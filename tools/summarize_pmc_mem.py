"""Summary of tools/pmc_mem.sh: medians per launch of the bounce traversal kernel's memory-pipeline and issue
counters, and the derived shares (per-CU busy fractions over the launch's cycles).
usage: python3 tools/summarize_pmc_mem.py --tag <tag>  ->  profiles/<tag>_pmc_mem.json"""
from __future__ import annotations

import argparse
import json
import pathlib
import statistics
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "tools"))
from summarize_pmc import dispatches  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", required=True)
    ap.add_argument("--kernel", default="k_trace_closest4d")
    a = ap.parse_args()
    src = ROOT / "gpurun_out" / "pmc_mem"
    c = {}
    for p in ("p1", "p2", "p3"):
        f = src / p / "run_counter_collection.csv"
        if not f.exists():
            continue
        ds = list(dispatches(f, a.kernel).values())
        for k in ds[0]:
            if k not in ("kernel",):
                c[k] = statistics.median(d[k] for d in ds)
    cyc = c["GRBM_GUI_ACTIVE"] / 8          # per XCD (GRBM sums the 8 XCDs)
    cus = 256
    out = {"kernel": a.kernel, "workload": "config-2 bounce rays (tools/trace_kernel_bench.py --set bounce)",
           "counters_per_launch_median": c,
           "launch_cycles": cyc,
           "ta_busy_frac": round(c["TA_TA_BUSY"] / (cus * cyc), 4) if "TA_TA_BUSY" in c else None,
           "td_busy_frac": round(c["TD_TD_BUSY"] / (cus * cyc), 4) if "TD_TD_BUSY" in c else None,
           "vmem_rd_insts": c.get("SQ_INSTS_VMEM_RD"), "lds_insts": c.get("SQ_INSTS_LDS"), "salu_insts": c.get("SQ_INSTS_SALU"),
           "tcp_wave_latency_cycles": round(c["TCP_TCP_LATENCY"] / c["TA_TCP_STATE_READ"], 1) if c.get("TA_TCP_STATE_READ") else None,
           "tcc_read_latency_cycles": round(c["TCP_TCC_READ_REQ_LATENCY"] / c["TCP_TCC_READ_REQ"], 1) if c.get("TCP_TCC_READ_REQ") else None,
           "l1_hit_frac": round(1 - c["TCP_TCC_READ_REQ"] / c["TCP_TOTAL_CACHE_ACCESSES"], 4) if c.get("TCP_TOTAL_CACHE_ACCESSES") and "TCP_TCC_READ_REQ" in c else None,
           "note": "TA/TD busy: per-CU cycles summed over the 256 CUs / (256 x launch cycles); TCP latency: "
                   "TCP_TCP_LATENCY / TA_TCP_STATE_READ (per wave instruction); L2 read latency: "
                   "TCP_TCC_READ_REQ_LATENCY / TCP_TCC_READ_REQ"}
    dst = ROOT / "profiles" / f"{a.tag}_pmc_mem.json"
    dst.write_text(json.dumps(out, indent=1) + "\n")
    print(json.dumps({k: v for k, v in out.items() if k != "counters_per_launch_median"}, indent=1))


if __name__ == "__main__":
    main()
