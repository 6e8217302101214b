#!/bin/bash
# round 4 GPU call: the whole -m gpu suite and smoke() on the final kernels
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r4y}
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?
echo "pytest_gpu.log rc=$rc"; tail -6 $O/pytest_gpu.log
if [ $rc -ge 124 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc2=$?
echo "smoke.log rc=$rc2"; tail -3 $O/smoke.log
exit $(( rc > rc2 ? rc : rc2 ))
