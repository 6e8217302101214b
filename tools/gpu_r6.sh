#!/bin/bash
# Round-6 GPU jobs, one per call: bash tools/gpu_r6.sh <job> [TAG]
# Every GPU step runs under its own limit; the job stops at the first failure.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
JOB=$1
O=gpurun_out/${2:-r6_$JOB}
mkdir -p $O
R=$GRAFT_REPO_ROOT
step() { local log=$1; shift; "$@" > $O/$log 2>&1; local rc=$?; echo "$log rc=$rc"; tail -${TAILN:-4} $O/$log; if [ $rc -ne 0 ]; then exit $rc; fi; }
PYT="python -u -m pytest -m gpu -q -rf --timeout 300 --timeout-method thread"
bench() { step bench$1.log timeout -k 10 300 python3 -u bench.py --steps ${STEPS:-30} --warmup 5 --no-cpu-baseline --no-secondary; }
trace() {
  step prof.log timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-secondary
  local f=$(find $O/prof -name '*kernel_trace.csv' | head -1)
  TAILN=${TRACEN:-60} step step.txt python3 tools/step_dump.py $f
  cp $O/prof/run_kernel_stats.csv $O/kernel_stats.csv 2>/dev/null; rm -rf $O/prof
}
case $JOB in
  watchdog)
    # capture fix: probe (drained), the whole trainer module, bench + trace; then the
    # un-drained probe LAST (the hypothesis is that it aborts)
    step probe_drained.log timeout -k 10 120 python3 -u tools/probe/capture_watchdog.py drained
    TAILN=8 step pytest_trainer.log timeout -k 10 900 $PYT tests/test_gpu_trainer.py
    bench
    trace
    TAILN=30 step probe_pending.log timeout -k 10 120 python3 -u tools/probe/capture_watchdog.py pending
    ;;
  tests)
    TAILN=8 step pytest.log timeout -k 10 900 $PYT ${TFILES:-tests} ${TK:+-k "$TK"}
    ;;
  smoke)
    step smoke.log timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()"
    ;;
  iter)
    [ -n "$TFILES" ] && TAILN=8 step pytest.log timeout -k 10 900 $PYT $TFILES ${TK:+-k "$TK"}
    bench
    [ -n "$TRACE" ] && trace
    ;;
  evidence)
    # the round's evidence tables on this tree (tools/gpu_evidence.sh: -m gpu suite, smoke, PMC traffic /
    # MFMA, rocprof families, kernel stats, the default bench line), then a 2-rank gloo rehearsal of the
    # data-parallel bench path (eager, ranks sharing the one GPU)
    TAG=${2:-r6ev} bash tools/gpu_evidence.sh || exit $?
    step gloo2.log env RNVP_BENCH_BACKEND=gloo timeout -k 10 600 python3 -u bench.py --gpus 2 --steps 2 --warmup 1 --no-secondary --no-cpu-baseline
    ;;
  ab)
    # library A/B: optional tests, the conv microbench cases ${MB} and the step, HEAD build vs $BASE
    [ -n "$TFILES" ] && TAILN=8 step pytest.log timeout -k 10 900 $PYT $TFILES ${TK:+-k "$TK"}
    # BASE: a library built from the SAME header revision (the binding refuses
    # another one: rnvp_struct_size); without it only the HEAD build runs
    [ -n "$MB" ] && TAILN=40 step mb_new.log timeout -k 10 300 python3 -u tools/conv_microbench.py $MB
    [ -n "$MB" ] && [ -n "$BASE" ] && TAILN=40 step mb_base.log env RNVP_LIB_PATH=$R/$BASE timeout -k 10 300 python3 -u tools/conv_microbench.py $MB
    [ -n "$STAMPS" ] && TAILN=40 step stamps.log timeout -k 10 300 python3 -u tools/probe/deep_stamps.py
    STEPS=${STEPS:-30} bench _new
    [ -n "$BASE" ] && step bench_base.log env RNVP_LIB_PATH=$R/$BASE timeout -k 10 300 python3 -u bench.py --steps ${STEPS:-30} --warmup 5 --no-cpu-baseline --no-secondary
    [ -n "$BASE" ] && STEPS=${STEPS:-30} bench _new2
    [ -n "$TRACE" ] && trace
    ;;
  *) echo "unknown job $JOB"; exit 2;;
esac
exit 0
