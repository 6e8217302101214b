#!/bin/bash
# GPU-box: conv parity, bench line, rocprofv3 kernel-trace stats of a short bench run.
mkdir -p gpurun_out
step() { local log=$1; shift; "$@" > gpurun_out/$log 2>&1; local rc=$?; echo "$log rc=$rc"; tail -2 gpurun_out/$log; if [ $rc -gt 1 ]; then exit $rc; fi; }
step t_conv.log timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py -x -q --timeout 120 --timeout-method thread
step bench.log timeout -k 10 300 python -u bench.py
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof.log 2>&1
echo "prof rc=$?"
