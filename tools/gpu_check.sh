#!/bin/bash
# GPU-box check: kernel parity, full GPU suite, conv microbench, bench line.
# Test failures (pytest exit 1) do not stop the script; faults/timeouts do.
mkdir -p gpurun_out
step() { local log=$1; shift; "$@" > gpurun_out/$log 2>&1; local rc=$?; echo "$log rc=$rc"; tail -3 gpurun_out/$log; if [ $rc -gt 1 ]; then exit $rc; fi; }
step t_conv.log timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py -x -q --timeout 120 --timeout-method thread
step t_gpu.log timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread
step mb.log timeout -k 10 300 python -u tools/conv_microbench.py --v01
step bench.log timeout -k 10 300 python -u bench.py
