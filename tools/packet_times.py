"""Per-wave timeline of the packet kernel from a -DLH2_TRACE_TIMES build (LH2_TRACE_TIMES_OUT dump):
start, when the wave took its last packet, end (100 MHz), packets per wave."""
import sys

import numpy as np

d = np.fromfile(sys.argv[1], dtype=np.uint64).reshape(-1, 4)
d = d[d[:, 2] > 0]
t0 = d[:, 0].min()
last, end = (d[:, 1] - t0) / 100.0, (d[:, 2] - t0) / 100.0
pk = d[:, 3].astype(np.int64)
print(f"waves {len(d)}  kernel span {end.max():.1f} us  packets {pk.sum()} (per wave median {np.median(pk):.0f}, max {pk.max()})")
print(f"last packet taken at: min {last.min():.1f}  median {np.median(last):.1f}  max {last.max():.1f} us")
print(f"wave end: min {end.min():.1f}  median {np.median(end):.1f}  p90 {np.percentile(end, 90):.1f}  max {end.max():.1f} us")
print(f"last packet duration: median {np.median(end - last):.1f}  p90 {np.percentile(end - last, 90):.1f}  max {(end - last).max():.1f} us")
