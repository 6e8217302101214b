cd $GRAFT_REPO_ROOT
O=gpurun_out/shards; mkdir -p $O
B="python3 -u bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-secondary"
for r in 1 2; do
  for v in base s16 s32; do
    if [ $v = base ]; then timeout -k 10 300 $B > $O/$v.$r.log 2>&1 || exit 1
    else RNVP_LIB_PATH=$GRAFT_REPO_ROOT/tools/variants/lib_$v.so timeout -k 10 300 $B > $O/$v.$r.log 2>&1 || exit 1; fi
    echo $v $r $(grep -o '"ms_per_step": [0-9.]*' $O/$v.$r.log) $(grep -o '"coupling": {"ms": [0-9.]*' $O/$v.$r.log)
  done
done
