#!/bin/bash
# round 4 GPU call: group members by value in the kernel arguments (global instead of flat memory ops),
# BN-table affine parameters preloaded in the band / s1 prologues.  No prev.so A/B: the library ABI of
# rnvp_net_group changed (host table), an older library would read a host pointer on the device.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r4ae}
mkdir -p $O
step() { local log=$1; shift; "$@" > $O/$log 2>&1; local rc=$?; echo "$log rc=$rc"; tail -${TAILN:-4} $O/$log; if [ $rc -ne 0 ]; then exit $rc; fi; }
TAILN=3 step pytest.log timeout -k 10 900 python -u -m pytest tests/test_gpu_group.py tests/test_gpu_conv.py tests/test_gpu_parity.py tests/test_gpu_trainer.py -m gpu -q -rf --timeout 300 --timeout-method thread
step ab.log env STEPS=30 VARIANTS="||" TAG=${TAG:-r4ae}/ab bash tools/gpu_ab.sh
step prof.log timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-secondary
