#!/bin/bash
# round 4 GPU call: packed BN+ReLU staging transform (wgrad / deep / band / stream / fan-out)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4x}
mkdir -p $O
step() { local log=$1; shift; "$@" > $O/$log 2>&1; local rc=$?; echo "$log rc=$rc"; tail -${TAILN:-4} $O/$log; if [ $rc -ne 0 ]; then exit $rc; fi; }
soft() { local log=$1; shift; "$@" > $O/$log 2>&1; local rc=$?; echo "$log rc=$rc"; tail -${TAILN:-4} $O/$log; if [ $rc -ge 124 ]; then exit $rc; fi; }
TAILN=6 soft pytest.log timeout -k 10 900 python -u -m pytest tests/test_gpu_conv.py -m gpu -q -rf --timeout 300 --timeout-method thread
TAILN=40 step mb.txt timeout -k 10 300 python3 -u tools/conv_microbench.py
step ab.log env STEPS=30 VARIANTS='||' TAG=${TAG:-r4x}/ab bash tools/gpu_ab.sh
