#!/bin/bash
# round 4, first GPU call: the new parity tests, the multi-rank launcher
# rehearsal (gloo, two ranks on the one GPU) and the default bench line
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4a}
mkdir -p $O
step() { local log=$1; shift; "$@" > $O/$log 2>&1; local rc=$?; echo "$log rc=$rc"; tail -${TAILN:-4} $O/$log; if [ $rc -ne 0 ]; then exit $rc; fi; }
step pytest_new.log timeout -k 10 600 python -u -m pytest tests/test_gpu_group.py tests/test_gpu_trainer.py -m gpu -v -rf --timeout 240 --timeout-method thread
step gloo2.log env RNVP_BENCH_BACKEND=gloo timeout -k 10 400 python3 -u bench.py --gpus 2 --steps 3 --warmup 1 --no-secondary --no-cpu-baseline
step bench.log timeout -k 10 600 python3 -u bench.py
