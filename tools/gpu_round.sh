# One GPU call: parity tests, smoke, bench, kernel-trace profile, PMC traffic passes.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
B="python3 bench.py --no-cpu-baseline --no-graph --steps 1 --warmup 1 --pmc-markers gpurun_out/markers.json"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof.log 2>&1 && \
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run -- $B > gpurun_out/pmc_fetch.log 2>&1 && \
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run -- $B > gpurun_out/pmc_write.log 2>&1 && \
python3 tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write gpurun_out/markers.json gpurun_out/pmc_traffic.json > gpurun_out/pmc_traffic.txt 2>&1 ; \
timeout -k 10 300 python bench.py --traffic gpurun_out/pmc_traffic.json > gpurun_out/bench.json 2> gpurun_out/bench.err
echo EXIT $?
