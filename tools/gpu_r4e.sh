#!/bin/bash
# round 4 GPU call: measurements first (microbench + step A/Bs of this
# round's changes, bench line, trace), then the parity suite of the changed
# areas.  A failing test does not stop the call; a timeout / abort / fault does.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4e}
mkdir -p $O
step() { local log=$1; shift; "$@" > $O/$log 2>&1; local rc=$?; echo "$log rc=$rc"; tail -${TAILN:-4} $O/$log; if [ $rc -ne 0 ]; then exit $rc; fi; }
soft() { local log=$1; shift; "$@" > $O/$log 2>&1; local rc=$?; echo "$log rc=$rc"; tail -${TAILN:-4} $O/$log; if [ $rc -ge 124 ]; then exit $rc; fi; }
step mb_band1.txt timeout -k 10 300 python3 -u tools/conv_microbench.py --case=3x3
step mb_band0.txt env RNVP_BAND2=0 timeout -k 10 300 python3 -u tools/conv_microbench.py --case=3x3
step mb_wt1.txt timeout -k 10 300 python3 -u tools/conv_microbench.py --case=wgrad
step mb_wt0.txt env RNVP_WT_POLICY=0 timeout -k 10 300 python3 -u tools/conv_microbench.py --case=wgrad
step ab.log env STEPS=30 VARIANTS='RNVP_BAND2=0 RNVP_WT_POLICY=0 RNVP_CHAIN_COUPLING=0|RNVP_BAND2=1|RNVP_BAND2=0|RNVP_WT_POLICY=0|RNVP_CHAIN_COUPLING=0|RNVP_BAND2=1' TAG=${TAG:-r4e}/ab bash tools/gpu_ab.sh
step prof.log timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-secondary
f=$(find $O/prof -name '*kernel_trace.csv' | head -1)
step step.txt python3 tools/step_dump.py $f
rm -f $f
step gloo2.log env RNVP_BENCH_BACKEND=gloo timeout -k 10 400 python3 -u bench.py --gpus 2 --steps 3 --warmup 1 --no-secondary --no-cpu-baseline
soft pytest_new.log timeout -k 10 700 python -u -m pytest tests/test_gpu_group.py tests/test_gpu_trainer.py tests/test_gpu_deep.py tests/test_gpu_c4.py -m gpu -v -rf --timeout 300 --timeout-method thread
soft smoke.log timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench.log timeout -k 10 600 python3 -u bench.py
