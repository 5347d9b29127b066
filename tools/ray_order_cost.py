"""Cost of reordering a bounce-ray stream on the GPU (VERDICT r3 #2's alternative): the key computation
(direction octant + 30-bit Morton code of the origin), torch.sort of the 64-bit keys (rocPRIM radix sort)
and the gather of the origin / direction float4 streams, for the config-2 bounce ray count.  Compare
with the traversal time saved, tools/trace_kernel_bench.py --set both (bounce vs bounce_sorted)."""
from __future__ import annotations

import json

import torch


def main(n=2_010_597, iters=20):
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(1)
    o = torch.rand((n, 4), device=dev, generator=g)
    d = torch.randn((n, 4), device=dev, generator=g)

    def spread(x):
        x = (x | (x << 16)) & 0x030000FF
        x = (x | (x << 8)) & 0x0300F00F
        x = (x | (x << 4)) & 0x030C30C3
        return (x | (x << 2)) & 0x09249249

    def reorder():
        q = (o[:, :3] * 1023).to(torch.int64).clamp_(0, 1023)
        m = (spread(q[:, 0]) << 2) | (spread(q[:, 1]) << 1) | spread(q[:, 2])
        octant = ((d[:, 0] < 0).to(torch.int64) << 2) | ((d[:, 1] < 0).to(torch.int64) << 1) | (d[:, 2] < 0).to(torch.int64)
        _, idx = torch.sort((octant << 30) | m)
        return o.index_select(0, idx), d.index_select(0, idx)

    for _ in range(3):
        reorder()
    torch.cuda.synchronize()
    res = {}
    for name, fn in (("keys+sort+gather", reorder),
                     ("sort_only", lambda: torch.sort(torch.randint(0, 1 << 33, (n,), device=dev, generator=g)))):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        res[name] = round(e0.elapsed_time(e1) / iters, 4)
    print(json.dumps({"rays": n, "ms": res}))


if __name__ == "__main__":
    main()
