"""Per-kernel mean duration (us) and calls per frame from rocprofv3 --kernel-trace kernel_trace.csv files, side by
side for several runs (tools/ab_kstats.sh output).  usage: python3 tools/kstats_compare.py <dir> [<dir> ...]"""
import collections
import csv
import glob
import sys

cols = []
for d in sys.argv[1:]:
    f = (glob.glob(f"{d}/**/run_kernel_trace.csv", recursive=True) + glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True))[0]
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        agg[r["Kernel_Name"][:48]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3)
    cols.append(agg)
names = sorted(set().union(*cols), key=lambda n: -sum(sum(c.get(n, [])) for c in cols))
print("%-48s" % "kernel" + "".join("%22s" % d.rstrip("/").split("/")[-1][:20] for d in sys.argv[1:]))
for n in names:
    print("%-48s" % n + "".join("%14.1f us x%5d" % (sum(c[n]) / len(c[n]), len(c[n])) if n in c else "%22s" % "-" for c in cols))
