"""profiles/<tag>_valu_rate.jsonl from tools/valu_rate's output (round 6 format: per-SIMD s_memtime spans, tools/valu_rate.hip)
and the probe's ISA (tools/valu_rate_isa.py, committed beside it as <tag>_valu_rate_isa.txt).

One line per instruction class and waves per SIMD with cycles per wave64 VALU instruction per SIMD (median over the 1,024
SIMDs).  The pinned classes issue 64 VALU instructions per loop iteration; the node-step mix's count per iteration is the
ISA's (its loop body's v_* instructions), so every number divides by instructions that were counted in the code that ran.

usage: python3 tools/valu_rate_summary.py --tag r06a [--src gpurun_out/r06probe/valu_rate.jsonl]
"""
from __future__ import annotations

import argparse
import json
import pathlib
import subprocess
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", required=True)
    ap.add_argument("--src", default=str(ROOT / "gpurun_out" / "r06probe" / "valu_rate.jsonl"))
    a = ap.parse_args()
    isa_path = ROOT / "profiles" / f"{a.tag}_valu_rate_isa.txt"
    subprocess.run([sys.executable, str(ROOT / "tools" / "valu_rate_isa.py"), "--out", str(isa_path)], check=True,
                   capture_output=True)
    isa = {}
    for line in open(isa_path):
        if line.startswith("{"):
            d = json.loads(line)
            isa[d["mode"]] = d
    out = []
    for line in open(a.src):
        if not line.strip().startswith("{"):
            continue
        r = json.loads(line)
        m = isa[r["mode"]]
        if r.get("insts_per_iter") is None:
            r["insts_per_iter"] = m["valu"]
            r["cycles_per_wave_inst"] = round(r["cycles_per_iter"] / m["valu"], 3)
        elif r["insts_per_iter"] != m["valu"]:
            raise SystemExit(f"{r['mode']}: the probe divides by {r['insts_per_iter']} but the ISA loop has {m['valu']} VALU")
        r["isa_loop"] = {k: m[k] for k in ("valu", "salu", "s_nop", "branch")}
        r["isa_valu_opcodes"] = m["valu_opcodes"]
        out.append(r)
    dst = ROOT / "profiles" / f"{a.tag}_valu_rate.jsonl"
    dst.write_text("".join(json.dumps(r) + "\n" for r in out))
    for r in out:
        if r["waves_per_simd"] == 8:
            print(f"{r['mode']:6s} 8 waves/SIMD: {r['cycles_per_wave_inst']:.3f} cycles per wave64 instruction ({', '.join(r['isa_valu_opcodes'])})")


if __name__ == "__main__":
    main()
