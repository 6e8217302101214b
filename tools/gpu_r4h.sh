#!/bin/bash
# round 4 GPU call: conflict-free LDS pitches (band / deep / halo / stream /
# fan-out kernels), one-launch weight-gradient groups: microbench, step,
# LDS-conflict counters of the band and deep kernels, parity of the changed kernels
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4h}
mkdir -p $O
step() { local log=$1; shift; "$@" > $O/$log 2>&1; local rc=$?; echo "$log rc=$rc"; tail -${TAILN:-4} $O/$log; if [ $rc -ne 0 ]; then exit $rc; fi; }
soft() { local log=$1; shift; "$@" > $O/$log 2>&1; local rc=$?; echo "$log rc=$rc"; tail -${TAILN:-4} $O/$log; if [ $rc -ge 124 ]; then exit $rc; fi; }
TAILN=40 step mb.txt timeout -k 10 300 python3 -u tools/conv_microbench.py
step ab.log env STEPS=30 VARIANTS='|RNVP_WT_SPLIT=1|' TAG=${TAG:-r4h}/ab bash tools/gpu_ab.sh
P2="SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
for c in "s2 3x3 64->64 pro+stats:k_conv_band" "s5 3x3 512->512 pro+stats:k_conv_deep" "wgrad s5 3x3 512:k_wgrad"; do
  cs=${c%%:*}; kn=${c##*:}; tag=$(echo $cs | tr -c 'a-z0-9' '_')
  step pmc_$tag.log timeout -s KILL 90 rocprofv3 --pmc $P2 --output-format csv -d $GRAFT_REPO_ROOT/$O/pmc_$tag/pmc1 -o run -- python3 $GRAFT_REPO_ROOT/tools/conv_microbench.py --case="$cs"
  step pmc_$tag.txt python3 tools/pmc_case.py $O/pmc_$tag $kn
done
soft pytest.log timeout -k 10 900 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_group.py tests/test_gpu_deep.py -m gpu -q -rf --timeout 300 --timeout-method thread
