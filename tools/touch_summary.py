"""Config 5's compulsory traffic per closest-hit launch (a lower bound beside the FETCH_SIZE upper bound).

Input: the stderr of config-5 frames rendered with the LH2_TOUCH diagnostic build (gpuab/touch, `make EXTRA=-DLH2_TOUCH`):
one "LH2_TOUCH {...}" line per closest-hit launch with the unique quantized BVH4 node records (64 B) and leaf triangle
records (48 B) the launch read (lh2_trace4d.inc, one bit per record).  Per launch:

  unique bytes U = node bytes + triangle bytes + paths x (32 B ray in + 16 B hit record out)
  DRAM lower bound = max(0, U - 288 MiB): at most the 256 MiB Infinity Cache plus the eight 4 MiB L2s can hold bytes from
  before the launch (or absorb its writes), everything else crosses the HBM interface at least once.

The paths of a launch are the frame's (primary: every path; bounce: the extension rays), taken from the bench's
config-5 ray counts.  Output: profiles/<tag>_config5_touch.json (bench.py's roofline_config5 reads its lower bound).

usage: python3 tools/touch_summary.py <touch stderr> <bench_configs config-5 JSON line file> --tag r06x
"""
from __future__ import annotations

import argparse
import json
import pathlib
import statistics

ROOT = pathlib.Path(__file__).resolve().parents[1]
CACHE_BYTES = (256 + 8 * 4) * 1048576


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("touch_log")
    ap.add_argument("bench_json")
    ap.add_argument("--tag", required=True)
    a = ap.parse_args()
    rows = [json.loads(l.split("LH2_TOUCH ", 1)[1]) for l in open(a.touch_log) if "LH2_TOUCH " in l]
    c5 = [json.loads(l) for l in open(a.bench_json) if l.strip().startswith("{")]
    c5 = [r for r in c5 if r.get("config") == "config5"][-1]
    rays = {1: c5["primary_rays"], 2: c5["bounce1_rays"]}
    out = {"workload": "config 5: 100 x 100k-triangle instanced meshes, per-frame TLAS, 1920x1080 8 spp",
           "method": "LH2_TOUCH build: one bit per quantized BVH4 node (64 B) and leaf triangle record (48 B) a closest-hit launch "
                     "reads; unique bytes U = nodes x 64 + triangle records x 48 + rays x (32 B in + 16 B out); DRAM lower bound "
                     "max(0, U - 288 MiB of Infinity Cache + L2)",
           "launches": []}
    by = {}
    for r in rows:
        by.setdefault(r["pathLength"], []).append(r)
    for pl, rs in sorted(by.items()):
        n = rays.get(pl)
        if n is None:
            continue
        nodes = statistics.median(r["node_bytes"] for r in rs)
        tris = statistics.median(r["tri_bytes"] for r in rs)
        u = nodes + tris + 48.0 * n
        out["launches"].append({"pathLength": pl, "kind": "primary" if pl == 1 else "bounce", "rays": n, "frames": len(rs),
                                "unique_node_bytes": nodes, "unique_tri_bytes": tris,
                                "scene_node_bytes": rs[0]["scene_nodes"] * 64, "scene_tri_bytes": rs[0]["scene_tri_records"] * 48,
                                "ray_stream_bytes": 48 * n, "unique_bytes": u, "dram_lower_bound_bytes": max(0.0, u - CACHE_BYTES)})
    dst = ROOT / "profiles" / f"{a.tag}_config5_touch.json"
    dst.write_text(json.dumps(out, indent=1) + "\n")
    print(json.dumps(out))


if __name__ == "__main__":
    main()
