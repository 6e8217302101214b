#!/bin/bash
# GPU box: the -m gpu suite file by file (failures do not stop the script;
# an abort / fault / time limit does), then a short bench line.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${TAG:-t}
step() { local log=$1; shift; "$@" > gpurun_out/$log 2>&1; local rc=$?; echo "$log rc=$rc"; tail -4 gpurun_out/$log; if [ $rc -gt 1 ]; then exit $rc; fi; }
PT="python -u -m pytest -v -rf --timeout 300 --timeout-method thread"
for f in ${FILES:-test_gpu_conv test_gpu_parity test_gpu_trainer test_gpu_deep}; do
  step ${TAG}_$f.log timeout -k 10 900 $PT tests/$f.py ${PTARGS}
done
if [ -z "$NOBENCH" ]; then
  step ${TAG}_bench.log timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 10 --warmup 3
fi
