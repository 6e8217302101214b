#!/bin/bash
# GPU box, one optimisation iteration: focused parity tests, conv microbench
# subset, bench line (no secondary numbers / CPU baseline) and a kernel-trace
# profile of a short bench.  Each step under its own limit; stops at the first
# fault/abort/timeout.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${TAG:-it}
step() { local log=$1; shift; "$@" > gpurun_out/$log 2>&1; local rc=$?; echo "$log rc=$rc"; tail -3 gpurun_out/$log; if [ $rc -gt 1 ]; then exit $rc; fi; }
step ${TAG}_pytest.log timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_conv.py} -m gpu -x -q --timeout 120 --timeout-method thread
if [ -n "$MB" ]; then
  step ${TAG}_mb.log timeout -k 10 300 python -u tools/conv_microbench.py $MB
fi
step ${TAG}_bench.log timeout -k 10 300 python -u bench.py --no-secondary --no-cpu-baseline ${BENCHARGS}
if [ -z "$NOPROF" ]; then
  export TMPDIR=/tmp
  step ${TAG}_prof.log timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-secondary
fi
