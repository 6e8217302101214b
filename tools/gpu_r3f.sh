O=gpurun_out/r3f; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_chain.py -m gpu -x -q -rf --timeout 200 --timeout-method thread -k "deep or chain or vs_float64" > $O/pytest.log 2>&1; echo pytest rc=$?; tail -3 $O/pytest.log
timeout -k 10 180 python3 -u tools/probe/deep_stamps.py > $O/stamps.txt 2>&1; cat $O/stamps.txt
timeout -k 10 300 python3 -u tools/conv_microbench.py --deep > $O/mb.txt 2>&1; tail -60 $O/mb.txt
TAG=r3f VARIANTS="RNVP_DEEP_MAXM3=4096|RNVP_DEEP_MAXM3=16384|RNVP_DEEP_MAXM1=4096|RNVP_DEEP_MAXM1=4096 RNVP_DEEP_MAXM3=16384" bash tools/gpu_ab.sh
