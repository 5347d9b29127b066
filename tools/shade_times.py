"""Summarise a -DLH2_SHADE_TIMES run (tools/shade_times.sh): k_shade's wave time between consecutive marks of shade_path."""
import json
import sys

NAMES = ["inputs: hit, instance, triangle, blue noise", "GetShadingData", "emission / alpha / flags",
         "RandomPointOnLight", "NEE: EvaluateBSDF + shadow ray", "SampleBSDF", "extension ray", "output compaction"]
line = open(sys.argv[1]).read().strip()
t = json.loads(line[line.index("["):])
tot = sum(t[:8])
for k in range(8):
    print(f"{k} {NAMES[k]:45s} {t[k] / tot:6.3f} of wave time   marks {t[8 + k]:>10d}   per mark {t[k] / max(1, t[8 + k]):8.1f} clk")
