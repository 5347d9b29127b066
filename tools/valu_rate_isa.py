"""The ISA behind tools/valu_rate (publish the probe's instructions).

Extracts the gfx950 code object from the built probe, disassembles it, finds each probe kernel's timed loop (the body
between the loop header and its backward branch) and counts its instructions by kind: VALU (v_*), SALU (s_* other than
s_nop / branches), s_nop, branches.  Writes the counts as JSON lines and the disassembled loop bodies as text, so the
instructions per iteration that tools/valu_rate divides by are checked against the code that ran.

usage: python3 tools/valu_rate_isa.py [--bin tools/valu_rate] --out profiles/r06_valu_rate_isa.txt
"""
from __future__ import annotations

import argparse
import json
import pathlib
import re
import subprocess
import tempfile

B = pathlib.Path("/opt/rocm/lib/llvm/bin")
ROOT = pathlib.Path(__file__).resolve().parents[1]


def disassemble(binary: pathlib.Path) -> str:
    with tempfile.TemporaryDirectory() as t:
        t = pathlib.Path(t)
        subprocess.run([B / "llvm-objcopy", f"--dump-section=.hip_fatbin={t / 'fat.bin'}", str(binary), str(t / "x")],
                       check=True)
        subprocess.run([B / "clang-offload-bundler", "--unbundle", "--type=o", f"--input={t / 'fat.bin'}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={t / 'k.co'}"], check=True)
        return subprocess.run([B / "llvm-objdump", "-d", "--no-show-raw-insn", str(t / "k.co")], check=True,
                              capture_output=True, text=True).stdout


def kernels(dis: str):
    """{kernel symbol: [(address, text)]}"""
    out, cur = {}, None
    for line in dis.splitlines():
        m = re.match(r"^([0-9a-f]+) <(.+)>:$", line)
        if m:
            cur = m.group(2)
            out[cur] = []
            continue
        m = re.match(r"^\s+([a-z_0-9]+.*?)\s*//\s*([0-9A-F]+):.*?(<[^>]*>)?$", line)
        if cur and m:
            out[cur].append((int(m.group(2), 16), m.group(1).strip() + (" " + m.group(3) if m.group(3) else "")))
    return out


def timed_loop(ins):
    """the innermost-to-outermost backward branch whose body holds the most VALU: the probe's timed loop"""
    best = None
    for i, (addr, txt) in enumerate(ins):
        tgt = None
        m2 = re.search(r"<\.?[^>]*\+0x([0-9a-f]+)>", txt)
        if txt.startswith("s_cbranch") and m2:
            tgt = int(m2.group(1), 16)
        if tgt is None:
            continue
        base = ins[0][0]
        tgt_abs = base + tgt if tgt < addr else tgt
        if tgt_abs >= addr:
            continue
        body = [x for x in ins if tgt_abs <= x[0] <= addr]
        nvalu = sum(1 for _, t in body if t.startswith("v_"))
        if best is None or nvalu > best[0]:
            best = (nvalu, body)
    return best[1] if best else []


def classify(body):
    c = {"valu": 0, "salu": 0, "s_nop": 0, "branch": 0, "other": 0}
    for _, t in body:
        op = t.split()[0]
        if op.startswith("v_"):
            c["valu"] += 1
        elif op == "s_nop":
            c["s_nop"] += 1
        elif op.startswith("s_cbranch") or op == "s_branch":
            c["branch"] += 1
        elif op.startswith("s_"):
            c["salu"] += 1
        else:
            c["other"] += 1
    return c


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bin", default=str(ROOT / "tools" / "valu_rate"))
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    ks = kernels(disassemble(pathlib.Path(a.bin)))
    lines, text = [], []
    for sym, ins in sorted(ks.items()):
        m = re.match(r"_Z\d+k_(\w+?)Pf", sym)
        if not m:
            continue
        body = timed_loop(ins)
        c = classify(body)
        ops = sorted({t.split()[0] for _, t in body if t.startswith("v_")})
        lines.append({"mode": m.group(1), "kernel": sym, "loop_instructions": len(body), **c, "valu_opcodes": ops})
        text.append(f"==== {sym}: timed loop, {len(body)} instructions ({json.dumps(c)})")
        text += [f"  {t}" for _, t in body]
    hdr = ("# tools/valu_rate's timed loops, disassembled from the gfx950 code object (tools/valu_rate_isa.py).\n"
           "# One JSON line per probe kernel (instruction counts per loop iteration), then each loop body.\n")
    pathlib.Path(a.out).write_text(hdr + "\n".join(json.dumps(x) for x in lines) + "\n\n" + "\n".join(text) + "\n")
    for x in lines:
        print(json.dumps({k: v for k, v in x.items() if k != "valu_opcodes"}))


if __name__ == "__main__":
    main()
