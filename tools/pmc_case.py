"""Per-dispatch averages of the PMC passes written by tools/gpu_pmc.sh, per
kernel name (substring filter).   python tools/pmc_case.py <dir> [name-filter]"""
import collections
import csv
import glob
import sys

d = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
for f in sorted(glob.glob(d + "/pmc*/**/*counter_collection.csv", recursive=True)):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        if flt not in n:
            continue
        agg[n][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[n].add(r.get("Dispatch_Id") or r.get("Correlation_Id"))
    for n, c in agg.items():
        k = len(disp[n])
        print(f.split("/")[-3] if "/" in f else f, n[:50], "dispatches", k)
        print("   " + "  ".join("%s %.4g" % (a, v / k) for a, v in sorted(c.items())))
