#!/bin/bash
# round 4 GPU call: same-box A/B of the previous library (abso/prev.so) against HEAD
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4ac}
mkdir -p $O
step() { local log=$1; shift; "$@" > $O/$log 2>&1; local rc=$?; echo "$log rc=$rc"; tail -${TAILN:-4} $O/$log; if [ $rc -ne 0 ]; then exit $rc; fi; }
P=RNVP_LIB_PATH=$GRAFT_REPO_ROOT/abso/prev.so
TAILN=40 step mb_prev.txt env $P timeout -k 10 300 python3 -u tools/conv_microbench.py
TAILN=40 step mb_head.txt timeout -k 10 300 python3 -u tools/conv_microbench.py
step ab.log env STEPS=30 VARIANTS="$P||$P|" TAG=${TAG:-r4ac}/ab bash tools/gpu_ab.sh
