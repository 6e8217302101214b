cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r5_pmc; mkdir -p $O
export RNVP_LIB_PATH=$PWD/tools/variants/lib_v0.so
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $PWD/$O/f -o run --output-format csv -- python3 tools/param_pass_bench.py 0 > $O/f.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $PWD/$O/w -o run --output-format csv -- python3 tools/param_pass_bench.py 0 > $O/w.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS -d $PWD/$O/s -o run --output-format csv -- python3 tools/param_pass_bench.py 0 > $O/s.log 2>&1 || exit 1
python3 - <<'PY'
import csv, glob, collections
for tag in ("f", "w", "s"):
    fs = glob.glob("gpurun_out/r5_pmc/%s/**/*counter_collection.csv" % tag, recursive=True)
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in fs:
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"][:40]
            agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, d in agg.items():
        print(tag, "%-40s" % k, " ".join("%s=%.4g" % (c, sum(v) / len(v)) for c, v in d.items()))
PY
rm -rf $O/f $O/w $O/s
