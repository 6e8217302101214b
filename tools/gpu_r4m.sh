#!/bin/bash
# round 4 GPU call: memory round-trip cost probe; BN-backward shard-first order
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4m}
mkdir -p $O
step() { local log=$1; shift; "$@" > $O/$log 2>&1; local rc=$?; echo "$log rc=$rc"; tail -${TAILN:-4} $O/$log; if [ $rc -ne 0 ]; then exit $rc; fi; }
soft() { local log=$1; shift; "$@" > $O/$log 2>&1; local rc=$?; echo "$log rc=$rc"; tail -${TAILN:-4} $O/$log; if [ $rc -ge 124 ]; then exit $rc; fi; }
TAILN=12 step latency.txt timeout -k 10 120 python3 -u tools/probe/latency_chain.py
TAILN=6 soft pytest.log timeout -k 10 600 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_parity.py -m gpu -q -rf --timeout 300 --timeout-method thread
step ab.log env STEPS=30 VARIANTS='||' TAG=${TAG:-r4m}/ab bash tools/gpu_ab.sh
