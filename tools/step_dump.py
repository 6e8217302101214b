"""Ordered dispatch list of the last complete training step in a rocprofv3
kernel trace: index, kernel, grid, duration, gap to the previous dispatch.

    python tools/step_dump.py run_results.db|kernel_trace.csv > step.txt

Also prints per-coupling totals grouped by scale (forward couplings start at
k_in_stats, backward ones at k_out_bwd_red) and the step's span/busy time."""
import sys
from collections import defaultdict

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from trace_summary import load_rows, short  # noqa: E402


def main():
    rows = load_rows(sys.argv[1])
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    adam = [i for i, r in enumerate(rows) if "k_adam" in r["Kernel_Name"]]
    seg = rows[adam[-2] + 1: adam[-1] + 1]
    prev_end = None
    busy = 0.0
    fam = defaultdict(lambda: [0, 0.0])
    for i, r in enumerate(seg):
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        d = (e - s) / 1e3
        gap = (s - prev_end) / 1e3 if prev_end is not None else 0.0
        prev_end = e
        busy += d
        g = "%sx%sx%s" % (r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"])
        n = short(r["Kernel_Name"])
        fam[n][0] += 1
        fam[n][1] += d
        print("%5d %-58s %-16s %8.2f %7.2f" % (i, n, g, d, gap))
    span = (int(seg[-1]["End_Timestamp"]) - int(seg[0]["Start_Timestamp"])) / 1e3
    print("# step: %d dispatches, span %.1f us, busy %.1f us" % (len(seg), span, busy))
    for n, (c, t) in sorted(fam.items(), key=lambda kv: -kv[1][1]):
        print("# %-58s %5d %9.1f %7.2f" % (n, c, t, t / c))


if __name__ == "__main__":
    main()
