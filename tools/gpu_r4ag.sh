#!/bin/bash
# round 4 GPU call: A/B of 32-channel deep tiles for the forward convs (RNVP_DEEP_FWD32)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4ag}
mkdir -p $O
step() { local log=$1; shift; "$@" > $O/$log 2>&1; local rc=$?; echo "$log rc=$rc"; tail -${TAILN:-4} $O/$log; if [ $rc -ne 0 ]; then exit $rc; fi; }
TAILN=12 step ab.log env STEPS=30 VARIANTS="|RNVP_DEEP_FWD32=1||RNVP_DEEP_FWD32=1" TAG=${TAG:-r4ag}/ab bash tools/gpu_ab.sh
