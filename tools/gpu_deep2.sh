#!/bin/bash
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${TAG:-d}
step() { local log=$1; shift; "$@" > gpurun_out/$log 2>&1; local rc=$?; echo "$log rc=$rc"; tail -2 gpurun_out/$log; if [ $rc -gt 1 ]; then exit $rc; fi; }
step ${TAG}_t_deep.log timeout -k 10 600 python -u -m pytest tests/test_gpu_conv.py -k "deep_family" -q --maxfail=20 --timeout 120 --timeout-method thread
step ${TAG}_stamps.log timeout -k 10 200 python -u tools/probe/deep_stamps.py
step ${TAG}_mb.log timeout -k 10 500 python -u tools/conv_microbench.py --deep --case=s3 --case=s4 --case=s5
for g in 2048 512 256; do
  RNVP_STREAM_GRID=$g step ${TAG}_mbs_$g.log timeout -k 10 200 python -u tools/conv_microbench.py --case=s1 --case=s2
done
step ${TAG}_pytest_gpu.log timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread
step ${TAG}_bench.log timeout -k 10 600 python -u bench.py --no-cpu-baseline --no-secondary
step ${TAG}_graphconc.log timeout -k 10 120 python -u tools/probe/graph_concurrency.py
step ${TAG}_bench_overlap.log timeout -k 10 600 python -u bench.py --no-cpu-baseline --no-secondary --overlap
