#!/bin/bash
# round 4 GPU call: weight gradient with the conflict-free k order (RNVP_WT_KO)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4q}
mkdir -p $O
step() { local log=$1; shift; "$@" > $O/$log 2>&1; local rc=$?; echo "$log rc=$rc"; tail -${TAILN:-4} $O/$log; if [ $rc -ne 0 ]; then exit $rc; fi; }
soft() { local log=$1; shift; "$@" > $O/$log 2>&1; local rc=$?; echo "$log rc=$rc"; tail -${TAILN:-4} $O/$log; if [ $rc -ge 124 ]; then exit $rc; fi; }
TAILN=8 soft pytest_wgrad.log timeout -k 10 600 python -u -m pytest tests/test_gpu_deep.py -m gpu -q -rf -k "grouped_wgrad or deep_coupling or trainer_config1_full_batch_bf16" --timeout 300 --timeout-method thread
TAILN=8 step mb_ko1.txt timeout -k 10 300 python3 -u tools/conv_microbench.py --case=wgrad
P2="SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
step pmc_ko1.log timeout -s KILL 90 rocprofv3 --pmc $P2 --output-format csv -d $GRAFT_REPO_ROOT/$O/pmc_ko1/pmc1 -o run -- python3 $GRAFT_REPO_ROOT/tools/conv_microbench.py --case="wgrad s1 3x3 32"
step pmc_ko1.txt python3 tools/pmc_case.py $O/pmc_ko1 k_wgrad
step ab.log env STEPS=30 VARIANTS='|' TAG=${TAG:-r4q}/ab bash tools/gpu_ab.sh
