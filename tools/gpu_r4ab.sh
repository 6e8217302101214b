#!/bin/bash
# round 4 GPU call: deep prologue without load branches (raw epilogue operands, unconditional table / bias loads)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4ab}
mkdir -p $O
step() { local log=$1; shift; "$@" > $O/$log 2>&1; local rc=$?; echo "$log rc=$rc"; tail -${TAILN:-4} $O/$log; if [ $rc -ne 0 ]; then exit $rc; fi; }
soft() { local log=$1; shift; "$@" > $O/$log 2>&1; local rc=$?; echo "$log rc=$rc"; tail -${TAILN:-4} $O/$log; if [ $rc -ge 124 ]; then exit $rc; fi; }
TAILN=3 soft pytest.log timeout -k 10 900 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_group.py -m gpu -q -rf --timeout 300 --timeout-method thread
TAILN=40 step mb.txt timeout -k 10 300 python3 -u tools/conv_microbench.py
step ab.log env STEPS=30 VARIANTS='||' TAG=${TAG:-r4ab}/ab bash tools/gpu_ab.sh
