"""profiles/<tag>_valu_rate.jsonl from tools/valu_rate_pmc.sh's output (gpurun_out/valu): one line per mode and
waves-per-SIMD with cycles per wave64 VALU instruction per SIMD.  The fma / pkfma counts are exact by
construction; the mix kernel's count is SQ_INSTS_VALU of its launches (median per launch, same block count:
the PMC pass runs the mix mode's four launch sizes in the same order, so launches are matched by grid size).
"""
from __future__ import annotations

import argparse
import collections
import csv
import json
import pathlib
import statistics

ROOT = pathlib.Path(__file__).resolve().parents[1]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", required=True)
    ap.add_argument("--src", default=str(ROOT / "gpurun_out" / "valu"))
    a = ap.parse_args()
    src = pathlib.Path(a.src)
    rows = [json.loads(x) for x in open(src / "rate.jsonl") if x.strip().startswith("{")]
    # SQ_INSTS_VALU per mix launch, keyed by grid size (work-items)
    per_grid = collections.defaultdict(list)
    csvs = list((src / "pmc").rglob("*counter_collection.csv"))
    if csvs:
        disp = collections.defaultdict(dict)
        for r in csv.DictReader(open(csvs[0])):
            if "k_mix" not in r["Kernel_Name"]:
                continue
            d = disp[int(r["Dispatch_Id"])]
            d["grid"] = int(r["Grid_Size"]) if r.get("Grid_Size") else None
            d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        mix = [r for r in rows if r["insts_per_iter"] is None]
        for i, (_, d) in enumerate(sorted(disp.items())):
            # without a grid column: the probe launches each size 11 times (1 untimed + 10), in order
            g = d["grid"] if d["grid"] is not None else mix[min(i // 11, len(mix) - 1)]["blocks"] * 256
            per_grid[g].append(d["SQ_INSTS_VALU"])
    out = []
    for r in rows:
        if r["insts_per_iter"] is None:
            grid = r["blocks"] * 256
            if grid not in per_grid:
                continue
            insts = statistics.median(per_grid[grid])
            cus = r["blocks"] // r["waves_per_simd"]
            per_simd = insts / (cus * 4.0)
            r = dict(r, insts_per_iter=round(insts / (r["blocks"] * 4 * r["iters"]), 2), sq_insts_valu=insts,
                     wave_insts_per_simd_per_cycle=round(per_simd / r["cycles_per_launch"], 4),
                     cycles_per_wave_inst=round(r["cycles_per_launch"] / per_simd, 3))
        out.append(r)
    dst = ROOT / "profiles" / f"{a.tag}_valu_rate.jsonl"
    dst.write_text("".join(json.dumps(r) + "\n" for r in out))
    for r in out:
        print(json.dumps(r))


if __name__ == "__main__":
    main()
