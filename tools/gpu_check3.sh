#!/bin/bash
# GPU box: full -m gpu suite, then the bench line (no CPU baseline / secondary numbers).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${TAG:-c}
step() { local log=$1; shift; "$@" > gpurun_out/$log 2>&1; local rc=$?; echo "$log rc=$rc"; tail -3 gpurun_out/$log; if [ $rc -gt 1 ]; then exit $rc; fi; }
step ${TAG}_pytest_gpu.log timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread
step ${TAG}_bench.log timeout -k 10 600 python -u bench.py --no-cpu-baseline --no-secondary
