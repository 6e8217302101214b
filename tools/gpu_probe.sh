#!/bin/bash
# GPU box (round 3): probes (launch floor, grid barrier, deep-conv phase
# stamps), then one build-measure iteration (tools/gpu_iter.sh: TESTS / PROF
# / MB as there).  Each step under its own limit; stops at the first failure.
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-it}
mkdir -p $O
if [ -z "$NOPROBE" ]; then
  timeout -k 10 60 tools/probe/launch_floor > $O/floor.txt 2>&1 || exit 1
  timeout -k 10 120 tools/probe/grid_barrier > $O/barrier.txt 2>&1 || exit 1
  cat $O/floor.txt $O/barrier.txt
  timeout -k 10 180 python3 -u tools/probe/deep_stamps.py > $O/stamps.txt 2>&1 || exit 1
  cat $O/stamps.txt
fi
bash tools/gpu_iter.sh
