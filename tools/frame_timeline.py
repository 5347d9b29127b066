"""Print one config-2 frame's kernel timeline (durations and launch gaps) from a rocprofv3
--kernel-trace CSV: the frame is the one starting at the median k_camera launch of the run.
Usage: python3 tools/frame_timeline.py gpurun_out/prof/stats/run_kernel_trace.csv"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
cams = [i for i, r in enumerate(rows) if r["Kernel_Name"].startswith("k_camera")]
k = len(cams) // 2
i0, i1 = cams[k], cams[k + 1]
prev = None
busy = 0
for r in rows[i0:i1 + 1]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev) / 1e3 if prev else 0.0
    print(f"{r['Kernel_Name'][:44]:44s} {(e - s) / 1e3:8.1f} us   gap {gap:6.1f}")
    if r is not rows[i1]:
        busy += e - s
    prev = e
frame = (int(rows[i1]["Start_Timestamp"]) - int(rows[i0]["Start_Timestamp"])) / 1e3
print(f"frame {frame:.1f} us, kernels {busy / 1e3:.1f} us, gaps {frame - busy / 1e3:.1f} us")
