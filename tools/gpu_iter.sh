#!/bin/bash
# GPU box: one build-measure iteration (round 3).  TESTS: pytest -k filter for
# the parity step; each step under its own limit, stop at the first failure.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-it}
O=gpurun_out/${TAG}
mkdir -p $O
step() { local log=$1; shift; "$@" > $O/$log 2>&1; local rc=$?; echo "$log rc=$rc"; tail -${TAILN:-4} $O/$log; if [ $rc -ne 0 ]; then exit $rc; fi; }
if [ -n "$TESTS" ]; then
  step pytest.log timeout -k 10 ${TTIME:-600} python -u -m pytest $TFILES -m gpu -x -q -rf --timeout 300 --timeout-method thread -k "$TESTS"
fi
if [ -n "$MB" ]; then
  step mb.txt timeout -k 10 300 python3 -u tools/conv_microbench.py "--case=$MB"
  if [ -n "$MB_OLD" ]; then step mb_old.txt env RNVP_WGRAD=0 timeout -k 10 300 python3 -u tools/conv_microbench.py "--case=$MB"; fi
fi
if [ -z "$NOBENCH" ]; then
  step bench.log timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-secondary
fi
if [ -n "$PROF" ]; then
  step prof.log timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-secondary
  f=$(find $O/prof -name '*kernel_trace.csv' | head -1)
  step step.txt python3 tools/step_dump.py $f
fi
