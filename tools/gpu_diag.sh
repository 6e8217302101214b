#!/bin/bash
# GPU box diagnostics (round 3): launch floor under the kernel trace, deep-family
# phase stamps, weight-gradient microbench + PMC passes.  Each step under its
# own limit; stops at the first failure.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-d}
O=gpurun_out/${TAG}
mkdir -p $O
step() { local log=$1; shift; "$@" > $O/$log 2>&1; local rc=$?; echo "$log rc=$rc"; tail -4 $O/$log; if [ $rc -ne 0 ]; then exit $rc; fi; }
step floor.txt timeout -k 10 60 tools/probe/launch_floor
step floor_trace.log timeout -k 10 90 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/floor_prof -o run -- $GRAFT_REPO_ROOT/tools/probe/launch_floor
step stamps.txt timeout -k 10 120 python3 -u tools/probe/deep_stamps.py
step mb_wgrad.txt timeout -k 10 120 python3 -u tools/conv_microbench.py --case=wgrad
CASE="${CASE:-wgrad s5 3x3}"
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD SQ_VALU_MFMA_BUSY_CYCLES"
P2="TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE"
P3="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_REQ_sum"
P4="SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
i=0
for P in "$P1" "$P2" "$P3" "$P4"; do
  i=$((i+1))
  step pmc$i.log timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d $GRAFT_REPO_ROOT/$O/pmc$i -o run -- python3 $GRAFT_REPO_ROOT/tools/conv_microbench.py "--case=$CASE"
done
