"""Per-family MFMA utilisation of the training step from one rocprofv3 --pmc
pass (SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE) over
``bench.py --pmc-markers <markers.json>`` (eager instrumented step, markers
around every engine launch).

    python tools/pmc_mfma.py <pmc_dir> <markers.json> [out.json]

MFMA busy % of a family = sum SQ_VALU_MFMA_BUSY_CYCLES / (sum GRBM_GUI_ACTIVE / 8
* 1024 SIMDs) * 100: rocprofv3's MfmaUtil (counter_defs.yaml, gfx950:
reduce(SQ_VALU_MFMA_BUSY_CYCLES,sum) / (reduce(GRBM_GUI_ACTIVE,max) * SIMD_NUM))
with GRBM_GUI_ACTIVE read as the sum over the 8 XCDs (MI355X_MICROARCH.md,
DVFS paragraph), summed over the family's dispatches."""
import json
import re
import sys
from collections import defaultdict

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from pmc_traffic import ENGINE, dispatches  # noqa: E402

SIMDS = 1024
XCDS = 8


def groups(ds, n_launch):
    idx = [i for i, (_, n, _) in enumerate(ds) if "k_marker" in n]
    idx = idx[-2 * n_launch:]
    if len(idx) != 2 * n_launch:
        raise SystemExit("found %d markers, expected %d" % (len(idx), 2 * n_launch))
    return [[(n, v) for _, n, v in ds[i0 + 1:i1] if ENGINE.search(n) and "k_marker" not in n]
            for i0, i1 in zip(idx[0::2], idx[1::2])]


def main():
    d, mfile = sys.argv[1:3]
    meta = json.load(open(mfile))
    fams = meta["families"]
    cnt = {c: groups(dispatches(d, c), len(fams))
           for c in ("SQ_VALU_MFMA_BUSY_CYCLES", "SQ_BUSY_CYCLES", "GRBM_GUI_ACTIVE")}
    agg = defaultdict(lambda: defaultdict(float))
    for c, gs in cnt.items():
        for f, g in zip(fams, gs):
            agg[f][c] += sum(v for _, v in g)
    for f in fams:
        agg[f]["launches"] = 0
    for f in fams:
        agg[f]["launches"] += 1
    adam = [(n, v) for _, n, v in dispatches(d, "SQ_VALU_MFMA_BUSY_CYCLES") if re.search(r"\bk_adam", n)]
    out = dict(config=meta.get("config"), stamp=meta.get("stamp"), formula="100 * MFMA_BUSY / (GRBM_GUI_ACTIVE / 8 * 1024)", families={})
    for f, a in sorted(agg.items(), key=lambda kv: -kv[1]["GRBM_GUI_ACTIVE"]):
        cyc = a["GRBM_GUI_ACTIVE"] / XCDS
        util = 100.0 * a["SQ_VALU_MFMA_BUSY_CYCLES"] / max(cyc * SIMDS, 1.0)
        out["families"][f] = dict(launches=int(a["launches"]), mfma_busy_pct=round(util, 3),
                                  mfma_busy_cycles=a["SQ_VALU_MFMA_BUSY_CYCLES"], gui_active=a["GRBM_GUI_ACTIVE"],
                                  sq_busy_cycles=a["SQ_BUSY_CYCLES"])
        print("%-12s launches %4d  MFMA busy %6.2f %%  (gui %.3g cycles/XCD)" % (f, a["launches"], util, cyc))
    if adam:
        print("calibration: k_adam (no MFMA) busy cycles", adam[-1][1])
    if len(sys.argv) > 3:
        json.dump(out, open(sys.argv[3], "w"), indent=1)


if __name__ == "__main__":
    main()
