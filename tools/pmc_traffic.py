"""Per-family HBM traffic per launch from rocprofv3 --pmc passes.

    python tools/pmc_traffic.py <fetch_dir> <write_dir> <markers.json> [out.json]

The passes are produced by (one counter set per run, see MI355X_MICROARCH.md
HBM section):

    rocprofv3 --pmc FETCH_SIZE -d <fetch_dir> -o run -- python3 bench.py --pmc-markers <markers.json> ...
    rocprofv3 --pmc WRITE_SIZE -d <write_dir> -o run -- python3 bench.py --pmc-markers <markers.json> ...

bench.py's instrumented step dispatches an empty ``k_marker`` before and
after every engine launch and writes the launch families in order to
markers.json; the engine kernels between the i-th pair of markers belong to
launch i.

Corrections (gfx950): FETCH_SIZE and WRITE_SIZE are reported in KiB;
FETCH_SIZE counts half the bytes of wide coalesced streaming reads, so it is
doubled.  The Adam kernel (k_adam, 16 B read + 12 B written per parameter, 1 B
mask) is reported beside the families as the calibration row.
"""
import csv
import glob
import json
import re
import sys
from collections import defaultdict

ENGINE = re.compile(r"\bk_\w+")


def dispatches(d, counter):
    """[(dispatch id, kernel name, value)] in dispatch order for one pass"""
    rows = {}
    for f in sorted(glob.glob(d + "/**/*.db", recursive=True)):     # rocpd SQLite (ROCm 7 default)
        import sqlite3
        q = "select dispatch_id, kernel_name, value from counters_collection where counter_name = ?"
        for did, name, v in sqlite3.connect(f).execute(q, (counter,)):
            n0, v0 = rows.get(did, (name, 0.0))
            rows[did] = (name, v0 + float(v))
    for f in sorted(glob.glob(d + "/**/*counter_collection.csv", recursive=True)):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            did = int(r.get("Dispatch_Id") or r.get("Correlation_Id"))
            name = r["Kernel_Name"]
            v = float(r["Counter_Value"])
            if did in rows:
                rows[did] = (name, rows[did][1] + v)
            else:
                rows[did] = (name, v)
    return [(k, n, v) for k, (n, v) in sorted(rows.items())]


def per_launch(ds, n_launch):
    """split the dispatches of the marked step into n_launch launch groups"""
    idx = [i for i, (_, n, _) in enumerate(ds) if "k_marker" in n]
    idx = idx[-2 * n_launch:]
    if len(idx) != 2 * n_launch:
        raise SystemExit("found %d markers, expected %d" % (len(idx), 2 * n_launch))
    groups = []
    for i0, i1 in zip(idx[0::2], idx[1::2]):
        g = [(n, v) for _, n, v in ds[i0 + 1:i1] if ENGINE.search(n) and "k_marker" not in n]
        groups.append(g)
    return groups


def main():
    fdir, wdir, mfile = sys.argv[1:4]
    out = sys.argv[4] if len(sys.argv) > 4 else None
    meta = json.load(open(mfile))
    fams = meta["families"]
    fd, wd = dispatches(fdir, "FETCH_SIZE"), dispatches(wdir, "WRITE_SIZE")
    fg, wg = per_launch(fd, len(fams)), per_launch(wd, len(fams))
    adam = None
    ar = [v for _, n, v in fd if re.search(r"\bk_adam", n)]
    aw = [v for _, n, v in wd if re.search(r"\bk_adam", n)]
    if ar and aw:   # last optimizer launch of the run
        adam = dict(read_bytes=ar[-1] * 2048.0, write_bytes=aw[-1] * 1024.0)
    agg = defaultdict(lambda: dict(launches=0, read=0.0, write=0.0, kernels=0))
    for fam, f, w in zip(fams, fg, wg):
        a = agg[fam]
        a["launches"] += 1
        a["kernels"] += len(f)
        a["read"] += sum(v for _, v in f) * 1024.0 * 2.0
        a["write"] += sum(v for _, v in w) * 1024.0
    res = dict(config=meta.get("config"), stamp=meta.get("stamp"), correction="bytes = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024", families={},
               adam_calibration=dict(measured=adam, n_params=meta.get("n_params")))
    alg = meta.get("alg_bytes", {})
    for fam, a in sorted(agg.items(), key=lambda kv: -kv[1]["read"] - kv[1]["write"]):
        tot = (a["read"] + a["write"]) / a["launches"]
        row = dict(launches=a["launches"], kernels=a["kernels"], read_per_launch=round(a["read"] / a["launches"]),
                   write_per_launch=round(a["write"] / a["launches"]), traffic_per_launch=round(tot))
        if fam in alg:
            row["alg_bytes_per_launch"] = round(alg[fam])
            row["traffic_over_alg"] = round(tot / max(alg[fam], 1.0), 3)
        res["families"][fam] = row
        print("%-14s launches %4d  read %10.0f  write %10.0f  per launch  (alg %s)" %
              (fam, a["launches"], a["read"] / a["launches"], a["write"] / a["launches"], row.get("alg_bytes_per_launch")))
    print("adam calibration:", adam, "params", meta.get("n_params"))
    if out:
        json.dump(res, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
