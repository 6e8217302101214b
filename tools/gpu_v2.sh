mkdir -p gpurun_out/v2
timeout -k 10 300 python -u -m pytest tests/test_gpu_deep.py -m gpu -x -q --timeout 200 --timeout-method thread -k wgrad > gpurun_out/v2/pytest.log 2>&1; rc=$?; tail -2 gpurun_out/v2/pytest.log; [ $rc -ne 0 ] && exit $rc
for v in 0 1 2; do if [ $v = 0 ]; then L=""; else L=$PWD/tools/probe/librealnvp_wt$v.so; fi; RNVP_LIB_PATH=$L timeout -k 10 120 python3 tools/conv_microbench.py --case=wgrad > gpurun_out/v2/mb$v.txt 2>&1 || exit 1; echo v$v; grep wgrad gpurun_out/v2/mb$v.txt; done
