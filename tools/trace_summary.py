"""Summarise a rocprofv3 --kernel-trace CSV per training step.

    python tools/trace_summary.py run_kernel_trace.csv|run_results.db [--by-shape] [--top N]

Steps are delimited by k_adam dispatches; the last complete step is reported
(kernel name, grid, LDS) with count, total and mean duration, plus the step's
wall span and the sum of kernel durations (gap = launch/idle time)."""
import argparse
import csv
import re
from collections import defaultdict


def short(name):
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    name = re.sub(r"unsigned short", "bf16", name)
    return re.sub(r"\(.*", "", name)[:60]


def load_rows(path):
    """rocprofv3 kernel-trace CSV, or the rocpd SQLite database (ROCm 7 default output)"""
    if not path.endswith(".db"):
        return list(csv.DictReader(open(path)))
    import sqlite3
    c = sqlite3.connect(path)
    q = ("select name, start, end, grid_x, grid_y, grid_z, lds_size from kernels")
    return [dict(Kernel_Name=n, Start_Timestamp=s, End_Timestamp=e, Grid_Size_X=gx, Grid_Size_Y=gy,
                 Grid_Size_Z=gz, LDS_Block_Size=lds) for n, s, e, gx, gy, gz, lds in c.execute(q)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--by-shape", action="store_true")
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    rows = load_rows(a.csv)
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    adam = [i for i, r in enumerate(rows) if "k_adam" in r["Kernel_Name"]]
    if len(adam) < 2:
        raise SystemExit("need >= 2 k_adam dispatches")
    seg = rows[adam[-2] + 1: adam[-1] + 1]
    t0 = int(seg[0]["Start_Timestamp"])
    t1 = int(seg[-1]["End_Timestamp"])
    agg = defaultdict(lambda: [0, 0.0])
    busy = 0.0
    for r in seg:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        busy += d
        k = short(r["Kernel_Name"])
        if a.by_shape:
            k += " g=%sx%sx%s lds=%s" % (r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"], r["LDS_Block_Size"])
        agg[k][0] += 1
        agg[k][1] += d
    print("step: %d dispatches, span %.3f ms, kernel busy %.3f ms" % (len(seg), (t1 - t0) / 1e6, busy / 1e3))
    print("%-100s %6s %10s %9s" % ("kernel", "n", "total_us", "mean_us"))
    for k, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:a.top]:
        print("%-100s %6d %10.1f %9.2f" % (k, n, t, t / n))


if __name__ == "__main__":
    main()
