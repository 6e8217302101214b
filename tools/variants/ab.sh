#!/bin/bash
# same-box step A/B over library variants built from the same header:
#   bash tools/variants/ab.sh TAG lib1.so lib2.so ...   ("-" = the in-tree build)
cd $GRAFT_REPO_ROOT; TAG=$1; shift
O=gpurun_out/$TAG; mkdir -p $O
for L in - "$@" -; do
  if [ "$L" = "-" ]; then E=""; else E="RNVP_LIB_PATH=$PWD/$L"; fi
  echo "[$L] $(env $E timeout -k 10 300 python3 -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-secondary 2>>$O/err.log | grep -o '"ms_per_step": [0-9.]*')" | tee -a $O/ab.log
  [ ${PIPESTATUS[0]} -eq 0 ] || exit 1
done
