"""Turn the scratch output of tools/profile_gpu.sh (gpurun_out/prof) into the committed summaries
under profiles/ for one round:

  profiles/<tag>_rocprof_kernel_stats.csv   rocprofv3 --kernel-trace --stats of bench.py
  profiles/<tag>_bench.json                 the bench.py JSON line of the same call
  profiles/<tag>_pmc_traffic.json           HBM bytes per roofline-kernel launch (the frame's
                                            diffuse bounce rays, bench.py's roofline kernel):
                                            2 x FETCH_SIZE (gfx950 calibration, MI355X_MICROARCH.md
                                            §HBM) + WRITE_SIZE, each from its own --pmc pass

bench.py reads bytes_per_launch from the newest *pmc_traffic*.json as roofline.traffic.
"""
from __future__ import annotations

import argparse
import csv
import json
import pathlib
import shutil
import statistics

ROOT = pathlib.Path(__file__).resolve().parents[1]


def _pmc(path, kernel):
    vals, durs = [], []
    for r in csv.DictReader(open(path)):
        if kernel in r["Kernel_Name"]:
            vals.append(float(r["Counter_Value"]))
            durs.append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    return vals, durs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", default="r01")
    ap.add_argument("--src", default=str(ROOT / "gpurun_out" / "prof"))
    ap.add_argument("--kernel", default="k_trace_closest4d", help="bench.py's roofline kernel (rocprof name)")
    a = ap.parse_args()
    src = pathlib.Path(a.src)
    dst = ROOT / "profiles"
    shutil.copy(src / "stats" / "run_kernel_stats.csv", dst / f"{a.tag}_rocprof_kernel_stats.csv")
    bench = json.loads((src / "bench.json").read_text().strip().splitlines()[-1])
    (dst / f"{a.tag}_bench.json").write_text(json.dumps(bench, indent=1) + "\n")

    kernel = a.kernel      # per-ray traversal (the packet kernel is k_trace_closest_packet)
    fetch, fd = _pmc(src / "pmc_fetch" / "run_counter_collection.csv", kernel)
    write, wd = _pmc(src / "pmc_write" / "run_counter_collection.csv", kernel)
    # kernel-trace durations of the roofline launches in the profiled bench run (the last kernel_iters)
    rows = [r for r in csv.DictReader(open(src / "stats" / "run_kernel_trace.csv")) if kernel in r["Kernel_Name"]]
    iters = 20
    trace_ms = statistics.mean(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows[-iters:]) / 1e6
    rays = bench["roofline"]["rays_per_launch"]
    fetch_b = 2.0 * statistics.median(fetch) * 1024.0      # FETCH_SIZE is in KiB; x2 per the gfx950 calibration
    write_b = statistics.median(write) * 1024.0
    out = {
        "kernel": f"{kernel} (config-2 bounce rays from the 1080p primary hits, tools/trace_kernel_bench.py --set bounce)",
        "rays_per_launch": rays,
        "fetch_size_kib_raw_median": statistics.median(fetch),
        "write_size_kib_median": statistics.median(write),
        "fetch_bytes": fetch_b, "write_bytes": write_b,
        "bytes_per_launch": fetch_b + write_b,
        "bytes_per_ray": (fetch_b + write_b) / rays,
        "algorithmic_bytes_per_ray": bench["roofline"]["hbm"]["model_bytes_per_ray"],
        "pmc_launch_ms_median": statistics.median(fd + wd) / 1e6,
        "rocprof_bench_roofline_launch_ms_mean": trace_ms,
        "bench_hip_event_launch_ms": bench["roofline"]["kernel_ms"],
        "note": "counters from two separate rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE); the BVH + "
                "triangle working set is L2/Infinity-Cache resident, so HBM bytes are ~ray + hit streams",
    }
    (dst / f"{a.tag}_pmc_traffic.json").write_text(json.dumps(out, indent=1) + "\n")
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
