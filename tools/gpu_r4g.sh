#!/bin/bash
# round 4 GPU call: band kernels' phase stamps + PMC, weight-gradient launch
# shapes, fan-out groups of the wide scales (parity + step A/B)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4g}
mkdir -p $O
step() { local log=$1; shift; "$@" > $O/$log 2>&1; local rc=$?; echo "$log rc=$rc"; tail -${TAILN:-4} $O/$log; if [ $rc -ne 0 ]; then exit $rc; fi; }
soft() { local log=$1; shift; "$@" > $O/$log 2>&1; local rc=$?; echo "$log rc=$rc"; tail -${TAILN:-4} $O/$log; if [ $rc -ge 124 ]; then exit $rc; fi; }
soft pytest_group.log timeout -k 10 400 python -u -m pytest tests/test_gpu_group.py -m gpu -v -rf --timeout 200 --timeout-method thread
TAILN=6 step band_stamps.txt timeout -k 10 200 python3 -u tools/probe/band_stamps.py
for v in 0 1; do
  i=0
  for P in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"; do
    i=$((i+1))
    step pmc_band${v}_$i.log env RNVP_BAND2=$v timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d $GRAFT_REPO_ROOT/$O/pmc_band$v/pmc$i -o run -- python3 $GRAFT_REPO_ROOT/tools/conv_microbench.py --case="s2 3x3 64->64 pro+stats"
  done
  step pmc_band$v.txt python3 tools/pmc_case.py $O/pmc_band$v k_conv_band
done
step mb_wt_split1.txt timeout -k 10 300 python3 -u tools/conv_microbench.py --case=wgrad
step mb_wt_split0.txt env RNVP_WT_SPLIT=0 timeout -k 10 300 python3 -u tools/conv_microbench.py --case=wgrad
step ab.log env STEPS=30 VARIANTS='RNVP_WT_SPLIT=0 RNVP_FANOUT=0|RNVP_WT_SPLIT=1 RNVP_FANOUT=0|RNVP_WT_SPLIT=1|RNVP_WT_SPLIT=0 RNVP_FANOUT=0|RNVP_WT_SPLIT=1' TAG=${TAG:-r4g}/ab bash tools/gpu_ab.sh
