#!/bin/bash
# GPU box: full -m gpu suite, smoke, default bench line.  Each step under its own limit; stops on fault/abort/timeout.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${TAG:-v}
step() { local log=$1; shift; "$@" > gpurun_out/$log 2>&1; local rc=$?; echo "$log rc=$rc"; tail -4 gpurun_out/$log; if [ $rc -gt 1 ]; then exit $rc; fi; }
step ${TAG}_pytest_gpu.log timeout -k 10 900 python -u -m pytest tests -m gpu -v -rf --timeout 300 --timeout-method thread ${PTARGS}
step ${TAG}_smoke.log timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()"
if [ -z "$NOBENCH" ]; then
  step ${TAG}_bench.log timeout -k 10 600 python -u bench.py ${BENCHARGS}
fi
