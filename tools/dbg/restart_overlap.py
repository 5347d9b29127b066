"""Diagnostic: overlapped restart frames vs serialised ones (room, path tail 2/3, shadowOverlap 0/1, earlyShade 0/1)."""
import sys, pathlib
sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[2]))
import numpy as np
import torch  # noqa: F401
from lighthouse2_amd import scene
from lighthouse2_amd.core import RenderCore

w, h = 128, 72
sc = scene.room_scene(40000, w, h)


def run(tail, sov, early, overlap, seq, warm):
    c = RenderCore(device=0)
    sc.load_into(c)
    c.set_target(w, h, 1)
    c.setting("maxPathLength", 4)
    c.setting("pathTail", tail)
    c.setting("shadowOverlap", sov)
    c.setting("earlyShade", early)
    c.setting("frameOverlap", overlap)
    for f in range(warm):
        sc.render_frame(c, converge=1 if f == 0 else 0)
        c.ray_counts()
    for conv in seq:
        sc.render_frame(c, converge=conv)
    a = c.accumulator()
    c.close()
    return a


for tail in (2, 3):
    for sov in (0, 1):
        for early in (0, 1):
            for seq in ((1,), (1, 0), (1, 0, 0), (0, 1)):
                a = run(tail, sov, early, 0, seq, 3)
                b = run(tail, sov, early, 1, seq, 3)
                d = float(np.linalg.norm(a[..., :3] - b[..., :3]) / max(np.linalg.norm(a[..., :3]), 1e-30))
                print(f"tail {tail} sov {sov} early {early} seq {seq}: rel {d:.3g} sums {a[..., :3].sum():.4g} {b[..., :3].sum():.4g} w-equal {np.array_equal(a[..., 3], b[..., 3])}", flush=True)
