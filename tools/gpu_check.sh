#!/bin/bash
# One gpurun call: GPU parity tests, a bench line, and a rocprofv3 kernel trace.
# Every GPU step has its own time limit and the chain stops at the first failure.
#   SKIP_TESTS=1  skip pytest;  PROF=<dir> add a rocprofv3 kernel-trace run
#   BENCH_ARGS / PROF_ARGS: arguments of the bench and of the profiled bench run
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 ${PYTEST_T:-600} python -m pytest tests -m gpu -x -q ${PYTEST_ARGS} > $OUT/pytest_gpu.log 2>&1
  rc=$?; echo "pytest_rc=$rc" >> $OUT/pytest_gpu.log
  [ $rc -ne 0 ] && exit $rc
fi
if [ -z "$SKIP_BENCH" ]; then
  timeout -k 10 ${BENCH_T:-400} python bench.py ${BENCH_ARGS:---steps 10 --warmup 3} > $OUT/bench.log 2>&1 || exit $?
fi
if [ -n "$PROF" ]; then
  cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/$PROF" -o run -- \
    python3 "$GRAFT_REPO_ROOT/bench.py" ${PROF_ARGS:---steps 5 --warmup 2 --no-cpu-baseline} > "$GRAFT_REPO_ROOT/$OUT/prof.log" 2>&1 || exit $?
fi
exit 0
