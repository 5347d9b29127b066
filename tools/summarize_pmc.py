"""Summaries of tools/pmc_round.sh (gpurun_out/pmc) committed under profiles/ for bench.py's roofline:

  profiles/<tag>_pmc_trace_sq.json       SQ issue counters of the dominant kernel, per launch (median
                                         over launches): VALU wave-instructions, VALU lane utilisation,
                                         effective clock (GRBM_GUI_ACTIVE / 8 XCDs / duration), and the
                                         VALU issue rate against the chip's VALU issue peak (1024
                                         SIMDs x 2.4 GHz / the cycles per wave64 VALU instruction that
                                         tools/valu_rate measured: the fastest of its mixes at 4-8 waves
                                         per SIMD, 3.58 for the node step's mix in round 3).
  profiles/<tag>_pmc_packet_sq.json      the same for the primary-ray packet launch.
  profiles/<tag>_pmc_config5_traffic.json  HBM bytes per launch of every kernel of config-5 frames
                                         (2 x FETCH_SIZE per the gfx950 calibration + WRITE_SIZE, KiB ->
                                         B), each from its own --pmc pass, and the achieved GB/s.
"""
from __future__ import annotations

import argparse
import collections
import csv
import json
import pathlib
import statistics

ROOT = pathlib.Path(__file__).resolve().parents[1]
SIMDS = 256 * 4
CLOCK_GHZ = 2.4


def cycles_per_valu():
    """SIMD cycles per wave64 VALU instruction of the fastest class tools/valu_rate measured at 8 waves per SIMD (round 6:
    the VOP2 fp32 add / multiply, 2.17; bench.py's roofline peak), else the guide's 2."""
    import glob
    files = sorted(glob.glob(str(ROOT / "profiles" / "*_valu_rate.jsonl")))
    if files:
        rows = [json.loads(x) for x in open(files[-1]) if x.strip().startswith("{")]
        rows = [r for r in rows if r.get("waves_per_simd") == 8 and r.get("cycles_per_wave_inst")]
        if rows:
            return min(r["cycles_per_wave_inst"] for r in rows)
    return 2.0


def dispatches(path, kernel=None):
    """{dispatch id: {"kernel", "ns", counter: value}} from a rocprofv3 counter_collection.csv."""
    out = collections.OrderedDict()
    for r in csv.DictReader(open(path)):
        if kernel and kernel not in r["Kernel_Name"]:
            continue
        d = out.setdefault(r["Dispatch_Id"], {"kernel": r["Kernel_Name"],
                                              "ns": int(r["End_Timestamp"]) - int(r["Start_Timestamp"])})
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return out


def med(ds, key):
    return statistics.median(d[key] for d in ds)


def trace_sq(src, kernel, p1="sq1", p2="sq2", what="config-2 bounce rays from the 1080p primary hits, tools/trace_kernel_bench.py --set bounce"):
    ds = list(dispatches(src / p1 / "run_counter_collection.csv", kernel).values())
    ds2 = list(dispatches(src / p2 / "run_counter_collection.csv", kernel).values()) if p2 else []
    ns = med(ds, "ns")
    valu = med(ds, "SQ_INSTS_VALU")
    # GRBM_GUI_ACTIVE counts the GPU's busy clocks over the counter pass's sampling window of the dispatch, summed over the 8
    # XCDs; for short launches (fills, k_finalize, k_shade: a few us) that window is longer than the kernel's own
    # timestamps and the quotient exceeds the chip's 2.4 GHz.  Only a clock the chip can run is kept;
    # otherwise the fields that divide by it are null (not evidence) and the issue fraction uses the nominal clock.  The raw
    # quotient is not published (it read 3.5-12.9 GHz for short launches)
    clk_raw = med(ds, "GRBM_GUI_ACTIVE") / 8 / ns      # GHz
    clk = clk_raw if 0.5 <= clk_raw <= 2.45 else None
    cycles = ns * (clk or CLOCK_GHZ)
    rate = valu / ns                                   # G wave-instructions / s
    cyc = cycles_per_valu()
    peak = SIMDS * CLOCK_GHZ / cyc
    counters = {k: med(ds, k) for k in ds[0] if k.startswith(("SQ_", "GRBM_"))}
    if ds2:
        counters.update({k: med(ds2, k) for k in ds2[0] if k.startswith("SQ_")})
    return {
        "kernel": f"{kernel} ({what})",
        "launches": len(ds), "launch_ms_median": ns / 1e6,
        "counters_per_launch_median": counters,
        "effective_clock_ghz": round(clk, 3) if clk else None,
        "valu_wave_insts_per_launch": valu,
        "valu_issue_rate_g_per_s": round(rate, 1),
        "valu_issue_peak_g_per_s": peak,
        "valu_issue_frac": round(rate / peak, 4),
        "valu_issue_frac_at_effective_clock": round(valu * cyc / (SIMDS * cycles), 4) if clk else None,
        "cycles_per_valu_instruction": cyc,
        "valu_lane_utilisation": round(counters["SQ_THREAD_CYCLES_VALU"] / (64 * counters["SQ_ACTIVE_INST_VALU"]), 4),
        "wave_cycles_waiting_frac": round(counters["SQ_WAIT_ANY"] / counters["SQ_WAVE_CYCLES"], 4)
        if "SQ_WAIT_ANY" in counters else None,
        "note": "VALU issue peak = 1024 SIMDs x 2.4 GHz / cycles per wave64 VALU instruction of the fastest class tools/valu_rate "
                "measured at 8 waves/SIMD (profiles/*_valu_rate.jsonl, round 6: VOP2 fp32 add / mul 2.17; VOP3 forms, fmac, "
                "max, compares and conversions ~4, the node step's mix 3.51); SQ_ACTIVE_INST_VALU counts one quad-cycle per VALU "
                "instruction whatever its issue cost (= SQ_INSTS_VALU on every probe class, profiles/r06b_valu_pmc/), so it is "
                "not a busy measure; SQ_WAVE_CYCLES and SQ_WAIT_* count quad-cycles (MI355X_MICROARCH.md)",
    }


def frame_sq(src, p1, p2, what):
    """Per kernel of a frame workload: the SQ issue summary of trace_sq (medians over that kernel's launches)."""
    names = sorted({d["kernel"] for d in dispatches(src / p1 / "run_counter_collection.csv").values()})
    rows = []
    for k in names:
        n = sum(1 for d in dispatches(src / p1 / "run_counter_collection.csv", k).values() if d["kernel"] == k)
        if n < 2:
            continue
        r = trace_sq(src, k, p1, p2, what)
        r["kernel"] = k
        rows.append(r)
    rows.sort(key=lambda r: -r["launch_ms_median"] * r["launches"])
    return {"workload": what, "kernels": rows}


def traffic(src, fetch, write, what):
    f = dispatches(src / fetch / "run_counter_collection.csv")
    w = dispatches(src / write / "run_counter_collection.csv")
    per = collections.defaultdict(lambda: {"fetch": [], "write": [], "ns": []})
    for d in f.values():
        per[d["kernel"]]["fetch"].append(2.0 * d["FETCH_SIZE"] * 1024.0)
        per[d["kernel"]]["ns"].append(d["ns"])
    for d in w.values():
        per[d["kernel"]]["write"].append(d["WRITE_SIZE"] * 1024.0)
        per[d["kernel"]]["ns"].append(d["ns"])
    rows = []
    for k, v in per.items():
        if len(v["fetch"]) < 3 or not v["write"]:
            continue
        b = statistics.median(v["fetch"]) + statistics.median(v["write"])
        ns = statistics.median(v["ns"])
        rows.append({"kernel": k, "launches": len(v["fetch"]), "bytes_per_launch": b,
                     "fetch_bytes": statistics.median(v["fetch"]), "write_bytes": statistics.median(v["write"]),
                     "launch_ms_median": ns / 1e6, "hbm_gb_s": round(b / ns, 1), "hbm_frac": round(b / ns / 8000.0, 4)})
    rows.sort(key=lambda r: -r["launch_ms_median"] * r["launches"])
    return {"workload": what,
            "kernels": rows,
            "note": "HBM bytes = 2 x FETCH_SIZE (gfx950 calibration) + WRITE_SIZE per launch (medians over "
                    "launches, separate --pmc passes); FETCH_SIZE also counts Infinity-Cache hits, so this "
                    "is an upper bound of DRAM traffic"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", required=True)
    ap.add_argument("--src", default=str(ROOT / "gpurun_out" / "pmc"))
    ap.add_argument("--kernel", default="k_trace_closest4d")
    a = ap.parse_args()
    src = pathlib.Path(a.src)
    dst = ROOT / "profiles"
    sq = trace_sq(src, a.kernel)
    (dst / f"{a.tag}_pmc_trace_sq.json").write_text(json.dumps(sq, indent=1) + "\n")
    print(json.dumps(sq, indent=1))
    if (src / "pk1").exists():
        pk = trace_sq(src, "k_trace_closest_packet", "pk1", None, "config-2 1080p primary rays in the frame's 8x8-tiled "
                                                                   "order, tools/trace_kernel_bench.py --set primary")
        (dst / f"{a.tag}_pmc_packet_sq.json").write_text(json.dumps(pk, indent=1) + "\n")
        print(json.dumps(pk, indent=1))
    C5 = "config 5: 100 x 100k-triangle instanced meshes, per-frame TLAS, 1920x1080 8 spp (tools/bench_configs.py --configs 5)"
    C3 = "config 3: 1M-triangle lit room, maxPathLength 4, 1920x1080 1 spp (tools/bench_configs.py --configs 3)"
    for tag, f, w, what in (("config5_traffic", "c5_fetch", "c5_write", C5), ("config3_traffic", "c3_fetch", "c3_write", C3)):
        if (src / f).exists() and (src / w).exists():
            t = traffic(src, f, w, what)
            (dst / f"{a.tag}_pmc_{tag}.json").write_text(json.dumps(t, indent=1) + "\n")
            print(json.dumps(t, indent=1))
    for tag, p1, p2, what in (("config5_sq", "c5_sq1", "c5_sq2", C5), ("config3_sq", "c3_sq1", "c3_sq2", C3)):
        if (src / p1).exists():
            t = frame_sq(src, p1, p2 if (src / p2).exists() else None, what)
            (dst / f"{a.tag}_pmc_{tag}.json").write_text(json.dumps(t, indent=1) + "\n")
            print(json.dumps(t, indent=1)[:2000])


if __name__ == "__main__":
    main()
