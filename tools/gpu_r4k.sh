#!/bin/bash
# round 4 GPU call: persistent band kernel with the static pipelined k-loop
# (RNVP_BAND2=1) vs the one-band kernel; then the coupling / BN-backward
# prefetch parity + step
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4k}
mkdir -p $O
step() { local log=$1; shift; "$@" > $O/$log 2>&1; local rc=$?; echo "$log rc=$rc"; tail -${TAILN:-4} $O/$log; if [ $rc -ne 0 ]; then exit $rc; fi; }
soft() { local log=$1; shift; "$@" > $O/$log 2>&1; local rc=$?; echo "$log rc=$rc"; tail -${TAILN:-4} $O/$log; if [ $rc -ge 124 ]; then exit $rc; fi; }
TAILN=20 soft pytest_band.log timeout -k 10 600 python -u -m pytest tests/test_gpu_conv.py -m gpu -q -rf -k "band or c1_full or s2_" --timeout 300 --timeout-method thread
TAILN=14 step mb_band1.txt timeout -k 10 300 python3 -u tools/conv_microbench.py --case=3x3
TAILN=14 step mb_band0.txt env RNVP_BAND2_TM64=4 timeout -k 10 300 python3 -u tools/conv_microbench.py --case=3x3
TAILN=6 step band_stamps.txt timeout -k 10 200 python3 -u tools/probe/band_stamps.py
step ab.log env STEPS=30 VARIANTS='|RNVP_BAND2_TM64=4|RNVP_BAND2=0|' TAG=${TAG:-r4k}/ab bash tools/gpu_ab.sh
