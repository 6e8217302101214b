#!/bin/bash
# GPU box, round evidence in one call (each step under its own limit, stops at
# the first failure):
#   1. the -m gpu suite and smoke()            (unless NOTEST=1)
#   2. PMC passes over one eager instrumented step, markers around every
#      engine launch: FETCH_SIZE, WRITE_SIZE (HBM traffic per family,
#      tools/pmc_traffic.py) and SQ_VALU_MFMA_BUSY_CYCLES / SQ_BUSY_CYCLES /
#      GRBM_GUI_ACTIVE (MFMA busy per family, tools/pmc_mfma.py)
#   3. a kernel trace of the graph-replayed step with captured markers
#      (per-family rocprof durations, tools/trace_families.py)
#   4. a kernel trace + stats of the plain bench (tools/step_dump.py)
#   5. the default bench line, fed the three family tables
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${TAG:-ev}
O=gpurun_out/$T
mkdir -p $O
# on exit keep the summaries and the step's kernel trace, drop the raw PMC /
# marker traces (gpurun copies back <= 64 MiB)
trap 'rm -rf $O/pmc_fetch $O/pmc_write $O/pmc_mfma $O/trace_fam; for f in kernel_stats kernel_trace; do [ -f $O/prof/run_$f.csv ] && cp $O/prof/run_$f.csv $O/$f.csv; done; rm -rf $O/prof' EXIT
step() { local log=$1; shift; "$@" > $O/$log 2>&1; local rc=$?; echo "$log rc=$rc"; tail -${TAILN:-3} $O/$log; if [ $rc -ne 0 ]; then exit $rc; fi; }
R=$GRAFT_REPO_ROOT
if [ -z "$NOTEST" ]; then
  step pytest_gpu.log timeout -k 10 1000 python -u -m pytest tests -m gpu -v -rf --timeout 300 --timeout-method thread
  step smoke.log timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()"
fi
B="python3 $R/bench.py --no-cpu-baseline --no-secondary --no-graph --steps 1 --warmup 1 --pmc-markers $R/$O/markers.json"
step pmc_fetch.log timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $R/$O/pmc_fetch -o run -- $B
step pmc_write.log timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $R/$O/pmc_write -o run -- $B
step pmc_mfma.log timeout -s KILL 150 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $R/$O/pmc_mfma -o run -- $B
step pmc_traffic.txt python3 tools/pmc_traffic.py $O/pmc_fetch $O/pmc_write $O/markers.json $O/pmc_traffic.json
step pmc_mfma.txt python3 tools/pmc_mfma.py $O/pmc_mfma $O/markers.json $O/pmc_mfma.json
step trace_fam.log timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/$O/trace_fam -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-secondary --graph-markers $R/$O/graph_markers.json
step rocprof_families.txt python3 tools/trace_families.py $(find $O/trace_fam -name "*kernel_trace.csv" | head -1) $O/graph_markers.json $O/rocprof_families.json
step prof.log timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-secondary
step step.txt python3 tools/step_dump.py $(find $O/prof -name "*kernel_trace.csv" | head -1)
step bench.log timeout -k 10 600 python -u bench.py --traffic $O/pmc_traffic.json --mfma $O/pmc_mfma.json --rocprof-families $O/rocprof_families.json
