"""Summarise the per-wave times of a -DLH2_TRACE_TIMES build (binary dump LH2_TRACE_TIMES_OUT):
how long the waves run before / after the work queue runs dry, and how the kernel's span is split."""
import sys

import numpy as np

d = np.fromfile(sys.argv[1], dtype=np.uint64).reshape(-1, 4)
d = d[d[:, 2] > 0]
t0 = d[:, 0].min()
start, exh, end = (d[:, 0] - t0) / 100.0, (d[:, 1] - t0) / 100.0, (d[:, 2] - t0) / 100.0   # 100 MHz -> us
it = (d[:, 3] & 0xffffffff).astype(np.int64)
dry = (d[:, 3] >> np.uint64(32)).astype(np.int64)
print(f"waves {len(d)}  kernel span {end.max():.1f} us")
print(f"queue exhausted at: min {exh.min():.1f}  median {np.median(exh):.1f}  max {exh.max():.1f} us")
print(f"wave end:           min {end.min():.1f}  median {np.median(end):.1f}  p90 {np.percentile(end, 90):.1f}  max {end.max():.1f} us")
print(f"tail per wave (end - exhausted): median {np.median(end - exh):.1f}  p90 {np.percentile(end - exh, 90):.1f}  max {(end - exh).max():.1f} us")
print(f"iterations per wave: median {np.median(it):.0f}, after exhaustion median {np.median(dry):.0f}; share after exhaustion {dry.sum() / it.sum():.2f}")
for q in (0.5, 0.9, 0.99, 1.0):
    print(f"  {q:4.2f} of the waves have ended by {np.quantile(end, q):.1f} us")
# the launch's drain: live waves over time after the first wave found the queue dry
ex0 = exh.min()
span = end.max()
print(f"drain (first queue-dry wave -> last wave end): {span - ex0:.1f} us = {(span - ex0) / span:.2f} of the span")
for f in (0.75, 0.5, 0.25, 0.1, 0.02):
    print(f"  {f:4.2f} of the waves still running at {np.quantile(end, 1 - f):.1f} us")
