#!/bin/bash
# round 4 final GPU call: the evidence tables of HEAD (tools/gpu_evidence.sh, NOTEST: the full -m gpu suite
# and smoke() passed on this tree in gpurun_out/r4y2), then an informational A/B (RNVP_DEEP_FWD32, default off)
cd $GRAFT_REPO_ROOT
TAG=r4ev NOTEST=1 bash tools/gpu_evidence.sh || exit $?
O=gpurun_out/r4ev
env STEPS=30 VARIANTS="|RNVP_DEEP_FWD32=1||RNVP_DEEP_FWD32=1" TAG=r4ev/ab bash tools/gpu_ab.sh > $O/ab_fwd32.log 2>&1
echo "ab_fwd32 rc=$?"; cat $O/ab_fwd32.log
