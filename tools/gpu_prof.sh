#!/bin/bash
# GPU box: launch-floor probe, rocprofv3 kernel trace of a short bench run, ordered dump of one step.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-p}
timeout -k 10 60 tools/probe/launch_floor > gpurun_out/${TAG}_launch_floor.txt 2>&1
echo "floor rc=$?"; tail -6 gpurun_out/${TAG}_launch_floor.txt
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-secondary ${BENCHARGS} > gpurun_out/${TAG}_prof.log 2>&1
rc=$?; echo "prof rc=$rc"; tail -2 gpurun_out/${TAG}_prof.log
[ $rc -ne 0 ] && exit $rc
f=$(find gpurun_out/${TAG}_prof -name '*kernel_trace.csv' | head -1)
python3 tools/step_dump.py $f > gpurun_out/${TAG}_step.txt 2>&1
echo "dump rc=$?"; tail -30 gpurun_out/${TAG}_step.txt
