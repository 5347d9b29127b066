"""Print one frame's kernel timeline (durations and gaps) from a rocprofv3 --kernel-trace CSV."""
import csv
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/quick/stats/run_kernel_trace.csv"
frame = int(sys.argv[2]) if len(sys.argv) > 2 else 8
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
ks = [(r["Kernel_Name"][:44], int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]
cams = [i for i, k in enumerate(ks) if k[0].startswith("k_camera")]
i0, i1 = cams[frame], cams[frame + 1]
t0, prev = ks[i0][1], ks[i0][1]
for name, s, e in ks[i0:i1 + 1]:
    print(f"{name:46s} {(e - s) / 1e3:9.1f} us  gap {(s - prev) / 1e3:6.1f}  at {(s - t0) / 1e3:8.1f}")
    prev = e
