#!/bin/bash
# GPU box, one call: -m gpu suite, smoke, default bench line, rocprofv3 kernel-trace stats of a short bench.
# Each step under its own limit; stops at the first fault/abort/timeout.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${TAG:-r2}
step() { local log=$1; shift; "$@" > gpurun_out/$log 2>&1; local rc=$?; echo "$log rc=$rc"; tail -3 gpurun_out/$log; if [ $rc -gt 1 ]; then exit $rc; fi; }
if [ -z "$NOTEST" ]; then
  step ${TAG}_pytest_gpu.log timeout -k 10 900 python -u -m pytest tests -m gpu -v -rf --timeout 300 --timeout-method thread ${PTARGS}
  step ${TAG}_smoke.log timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()"
fi
step ${TAG}_bench.log timeout -k 10 600 python -u bench.py ${BENCHARGS}
if [ -z "$NOPROF" ]; then
  export TMPDIR=/tmp
  step ${TAG}_prof.log timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-secondary
fi
