#!/bin/bash
# GPU box, end-of-round evidence in one call: the -m gpu suite, smoke, the
# default bench line (secondary numbers + CPU baseline), a rocprofv3 kernel
# trace of a short bench, and the two PMC passes (FETCH_SIZE / WRITE_SIZE,
# separate runs) attributed per kernel family by tools/pmc_traffic.py.  Each
# step under its own limit; stops at the first failure.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-final}
O=gpurun_out/${TAG}
step() { local log=$1; shift; "$@" > gpurun_out/$log 2>&1; local rc=$?; echo "$log rc=$rc"; tail -3 gpurun_out/$log; if [ $rc -ne 0 ]; then exit $rc; fi; }
if [ -z "$NOTEST" ]; then
  step ${TAG}_pytest_gpu.log timeout -k 10 900 python -u -m pytest tests -m gpu -v -rf --timeout 300 --timeout-method thread
  step ${TAG}_smoke.log timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()"
fi
B="python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-secondary --no-graph --steps 1 --warmup 1 --pmc-markers $GRAFT_REPO_ROOT/${O}_markers.json"
step ${TAG}_pmc_fetch.log timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $GRAFT_REPO_ROOT/${O}_pmc_fetch -o run -- $B
step ${TAG}_pmc_write.log timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $GRAFT_REPO_ROOT/${O}_pmc_write -o run -- $B
step ${TAG}_pmc_traffic.txt python3 tools/pmc_traffic.py ${O}_pmc_fetch ${O}_pmc_write ${O}_markers.json ${O}_pmc_traffic.json
step ${TAG}_prof.log timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/${O}_prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-secondary --traffic $GRAFT_REPO_ROOT/${O}_pmc_traffic.json
step ${TAG}_bench.log timeout -k 10 600 python -u bench.py --traffic ${O}_pmc_traffic.json
