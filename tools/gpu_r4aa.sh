#!/bin/bash
# round 4 GPU call: DPP row reductions in the coupling passes; step trace
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4aa}
mkdir -p $O
step() { local log=$1; shift; "$@" > $O/$log 2>&1; local rc=$?; echo "$log rc=$rc"; tail -${TAILN:-4} $O/$log; if [ $rc -ne 0 ]; then exit $rc; fi; }
soft() { local log=$1; shift; "$@" > $O/$log 2>&1; local rc=$?; echo "$log rc=$rc"; tail -${TAILN:-4} $O/$log; if [ $rc -ge 124 ]; then exit $rc; fi; }
TAILN=6 soft pytest.log timeout -k 10 900 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_parity.py -m gpu -q -rf --timeout 300 --timeout-method thread
step ab.log env STEPS=30 VARIANTS='||' TAG=${TAG:-r4aa}/ab bash tools/gpu_ab.sh
step prof.log timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-secondary
f=$(find $O/prof -name '*kernel_trace.csv' | head -1)
TAILN=75 step step.txt python3 tools/step_dump.py $f
rm -f $f
