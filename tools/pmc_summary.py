"""Average PMC counters per kernel from rocprofv3 --pmc CSV passes.

    python tools/pmc_summary.py <dir-with-p1,p2,...> [kernel-substring]"""
import csv
import glob
import sys
from collections import defaultdict


def main():
    d = sys.argv[1]
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    agg = defaultdict(lambda: defaultdict(list))
    for f in sorted(glob.glob(d + "/p*/run_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if filt and filt not in k:
                continue
            agg[k[:70]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in agg.items():
        print(k)
        for c, v in sorted(cs.items()):
            print("   %-36s %14.1f  (n=%d)" % (c, sum(v) / len(v), len(v)))


if __name__ == "__main__":
    main()
