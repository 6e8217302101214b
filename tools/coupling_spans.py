"""Per-coupling kernel time of one training step from a rocprofv3 kernel trace.

    python tools/coupling_spans.py run_results.db|kernel_trace.csv

Forward couplings start at k_in_stats, backward couplings at k_out_bwd_red;
the last complete step (between two k_adam dispatches) is reported: number of
dispatches and summed kernel duration per coupling, forward and backward."""
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from trace_summary import load_rows  # noqa: E402


def main():
    rows = load_rows(sys.argv[1])
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    adam = [i for i, r in enumerate(rows) if "k_adam" in r["Kernel_Name"]]
    seg = rows[adam[-2] + 1: adam[-1] + 1]
    groups, cur = [], None
    for r in seg:
        n = r["Kernel_Name"]
        if "k_in_stats" in n or "k_out_bwd_red" in n:
            cur = ["fwd" if "k_in_stats" in n else "bwd", 0, 0.0, int(r["Grid_Size_X"])]
            groups.append(cur)
        if cur is None:
            continue
        cur[1] += 1
        cur[2] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    tot = {"fwd": 0.0, "bwd": 0.0}
    for i, (k, n, us, g) in enumerate(groups):
        tot[k] += us
        print("%3d %s n=%3d %8.1f us  (first grid %d)" % (i, k, n, us, g))
    print("fwd total %.1f us, bwd total %.1f us" % (tot["fwd"], tot["bwd"]))


if __name__ == "__main__":
    main()
