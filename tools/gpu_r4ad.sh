#!/bin/bash
# round 4 GPU call: BN-backward apply with every prologue load issued in one batch; same-box A/B against abso/prev.so
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4ad}
mkdir -p $O
step() { local log=$1; shift; "$@" > $O/$log 2>&1; local rc=$?; echo "$log rc=$rc"; tail -${TAILN:-4} $O/$log; if [ $rc -ne 0 ]; then exit $rc; fi; }
soft() { local log=$1; shift; "$@" > $O/$log 2>&1; local rc=$?; echo "$log rc=$rc"; tail -${TAILN:-4} $O/$log; if [ $rc -ge 124 ]; then exit $rc; fi; }
P=RNVP_LIB_PATH=$GRAFT_REPO_ROOT/abso/prev.so
TAILN=3 soft pytest.log timeout -k 10 900 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_parity.py -m gpu -q -rf --timeout 300 --timeout-method thread
step ab.log env STEPS=30 VARIANTS="$P||$P|" TAG=${TAG:-r4ad}/ab bash tools/gpu_ab.sh
