cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r5_pp
for i in 0 1 2 3 4; do echo "== v$i" >> gpurun_out/r5_pp/pp.log; RNVP_LIB_PATH=$PWD/tools/variants/lib_v$i.so timeout -k 10 200 python3 -u tools/param_pass_bench.py 0 7 >> gpurun_out/r5_pp/pp.log 2>&1 || exit 1; done
cat gpurun_out/r5_pp/pp.log
