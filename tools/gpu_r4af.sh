#!/bin/bash
# round 4 GPU call: A/B of the s1 stream kernel's tiles per wave (RNVP_S1_TPW)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4af}
mkdir -p $O
step() { local log=$1; shift; "$@" > $O/$log 2>&1; local rc=$?; echo "$log rc=$rc"; tail -${TAILN:-4} $O/$log; if [ $rc -ne 0 ]; then exit $rc; fi; }
TAILN=12 step ab.log env STEPS=30 VARIANTS="|RNVP_S1_TPW=2|RNVP_S1_TPW=4||RNVP_S1_TPW=2|RNVP_S1_TPW=4" TAG=${TAG:-r4af}/ab bash tools/gpu_ab.sh
