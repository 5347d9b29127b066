"""The shade kernels' closed-form RandomBarycentrics (lighthouse2_amd/csrc/lh2_bary.h) against the reference's 16-level
subdivision loop (lights_shared.h:145-164, restated in tools/bary_check.cpp as the oracle restates it): bit-identical
(rx, ry, 1 - rx - ry) over a strided sweep of the 2^32 digit strings plus the strings of two equal-digit runs.  The full
sweep (stride 1, ~6 min on one core) was run when the closed form was introduced: 0 of 4294967569 mismatched."""
import json
import pathlib
import subprocess

ROOT = pathlib.Path(__file__).resolve().parents[1]


def test_closed_form_barycentrics_match_the_reference_loop(tmp_path):
    exe = tmp_path / "bary_check"
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", str(ROOT / "tools" / "bary_check.cpp"), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe), "1021"], check=True, capture_output=True, text=True).stdout
    res = json.loads(out.strip().splitlines()[-1])
    assert res["mismatches"] == 0 and res["checked"] > 4_000_000
