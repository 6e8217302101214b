#!/bin/bash
# GPU-box: conv parity, then microbench of the given cases/variants, then bench.
mkdir -p gpurun_out
step() { local log=$1; shift; "$@" > gpurun_out/$log 2>&1; local rc=$?; echo "$log rc=$rc"; tail -2 gpurun_out/$log; if [ $rc -gt 1 ]; then exit $rc; fi; }
step t_conv.log timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py -x -q --timeout 120 --timeout-method thread
step mb.log timeout -k 10 300 python -u tools/conv_microbench.py "$@"
step bench.log timeout -k 10 300 python -u bench.py --no-cpu-baseline
