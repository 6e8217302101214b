cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/wgdiag
for L in - tools/variants/lib_nosplit.so tools/variants/lib_noalias.so tools/variants/lib_nosplit_noalias.so; do
  if [ "$L" = "-" ]; then E=""; else E="RNVP_LIB_PATH=$PWD/$L"; fi
  echo "== $L"
  env $E timeout -k 10 200 python -u -m pytest -m gpu -q -s --timeout 120 --timeout-method thread tests/test_gpu_deep.py -k mixed > gpurun_out/wgdiag/$(basename $L).log 2>&1
  rc=$?; grep -E "^\[\(|passed|failed" gpurun_out/wgdiag/$(basename $L).log; [ $rc -le 1 ] || exit $rc
done
