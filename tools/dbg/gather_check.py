"""Debug helper (round 6): tests/test_gpu_multidevice.py::test_gather_ordering_under_a_lagging_device0 as a script that
prints every frame's rel-L2 against the one-device core, for whichever library LH2_CORE_LIB names, with and without the
gather stall and the deviceCount."""
import json
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from lighthouse2_amd import scene  # noqa: E402
from lighthouse2_amd.core import RenderCore  # noqa: E402


def rel_l2(a, b):
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def run(devices, stall, frames=4, w=160, h=96):
    sc = scene.room_scene(30000, w, h)
    c = RenderCore(device=0)
    try:
        if devices > 1:
            c.setting("deviceCount", devices)
            c.setting("gatherStallUs", stall)
        c.setting("maxPathLength", 4)
        sc.load_into(c)
        c.set_target(w, h, 1)
        bufs = [torch.zeros((h, w, 4), dtype=torch.float32, device="cuda") for _ in range(frames)]
        torch.cuda.synchronize()
        for f in range(frames):
            sc.render_frame(c, converge=1 if f == 0 else 0)
            c.copy_frame_async(bufs[f].data_ptr())
        c.sync()
        return [b.cpu().numpy() for b in bufs]
    finally:
        c.close()


def main():
    sc = scene.room_scene(30000, 160, 96)
    ref = []
    c = RenderCore(device=0)
    c.setting("maxPathLength", 4)
    sc.load_into(c)
    c.set_target(160, 96, 1)
    for f in range(4):
        sc.render_frame(c, converge=1 if f == 0 else 0)
        ref.append(c.frame())
    c.close()
    for devices, stall in ((1, 0), (3, 0), (3, 30000)):
        got = run(devices, stall)
        print(json.dumps({"devices": devices, "stall_us": stall,
                          "rel_l2": [round(rel_l2(g[..., :3], r[..., :3]), 8) for g, r in zip(got, ref)]}), flush=True)


if __name__ == "__main__":
    main()
