"""Kernel intervals of a few steady-state frames from a rocprofv3 --kernel-trace CSV, relative to the start of the
median frame's primary launch (k_trace_primary_packet, or k_camera): start, end, duration per kernel, so launches that
overlap (frameOverlap, the shadow side stream) show as overlapping intervals.
usage: python3 tools/overlap_timeline.py run_kernel_trace.csv [frames]"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
nf = int(sys.argv[2]) if len(sys.argv) > 2 else 2
starts = [i for i, r in enumerate(rows) if r["Kernel_Name"].startswith(("k_trace_primary_packet", "k_camera"))]
k = int(sys.argv[3]) if len(sys.argv) > 3 else len(starts) // 2
i0, i1 = starts[k], starts[min(k + nf, len(starts) - 1)]
t0 = int(rows[i0]["Start_Timestamp"])
for r in rows[i0:i1 + 1]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"{r['Kernel_Name'][:40]:40s} {(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f} us")
print(f"{nf} frames: {(int(rows[i1]['Start_Timestamp']) - t0) / 1e3 / nf:.1f} us per frame")
