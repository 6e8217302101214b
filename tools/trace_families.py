"""Per-family kernel durations of the graph-replayed training step, from a
rocprofv3 --kernel-trace of ``bench.py --graph-markers <markers.json>``
(the markers are captured into the step's graph: an empty k_marker before and
after every engine launch, families listed in markers.json in launch order).

    python tools/trace_families.py <kernel_trace.csv|results.db> <markers.json> [out.json]

For the last complete replayed step: per family the number of launches, the
sum and mean of the rocprof durations of the engine kernels between each
marker pair (a launch may be several kernels, e.g. split-K + its reduce).
bench.py puts the dominant family's mean beside its HIP-event figure
(roofline.rocprof_avg_launch_us)."""
import json
import sys
from collections import defaultdict

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from trace_summary import load_rows  # noqa: E402


def main():
    rows = load_rows(sys.argv[1])
    meta = json.load(open(sys.argv[2]))
    fams = meta["families"]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    adam = [i for i, r in enumerate(rows) if "k_adam" in r["Kernel_Name"]]
    if len(adam) < 2:
        raise SystemExit("need two complete steps in the trace")
    # the last complete step that carries the captured markers (bench.py's
    # instrumented eager step for the HIP-event roofline runs after the
    # replays, without them)
    seg, mk = None, []
    for j in range(len(adam) - 1, 0, -1):
        cand = rows[adam[j - 1] + 1: adam[j] + 1]
        mk = [i for i, r in enumerate(cand) if "k_marker" in r["Kernel_Name"]]
        if len(mk) == 2 * len(fams):
            seg = cand
            break
    if seg is None:
        raise SystemExit("no step with the %d captured markers in the trace" % (2 * len(fams)))
    agg = defaultdict(lambda: dict(launches=0, kernels=0, us=0.0))
    for f, i0, i1 in zip(fams, mk[0::2], mk[1::2]):
        a = agg[f]
        a["launches"] += 1
        for r in seg[i0 + 1:i1]:
            a["kernels"] += 1
            a["us"] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    out = dict(config=meta.get("config"), stamp=meta.get("stamp"), source="rocprofv3 kernel trace, graph-replayed step", families={})
    for f, a in sorted(agg.items(), key=lambda kv: -kv[1]["us"]):
        out["families"][f] = dict(launches=a["launches"], kernels=a["kernels"], total_ms=round(a["us"] / 1e3, 3),
                                  avg_launch_us=round(a["us"] / a["launches"], 2))
        print("%-12s launches %4d kernels %4d total %8.3f ms avg %7.2f us" % (
            f, a["launches"], a["kernels"], a["us"] / 1e3, a["us"] / a["launches"]))
    if len(sys.argv) > 3:
        json.dump(out, open(sys.argv[3], "w"), indent=1)


if __name__ == "__main__":
    main()
