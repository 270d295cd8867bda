# Round-3 GPU job: full -m gpu suite (no -x: every failure listed), smoke, bench.
# usage: tools/jobs/r3_run.sh TAG [pytest args...]
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
tag=$1; shift
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest ${@:-tests} -m gpu -q -rfE --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_$tag.log 2>&1
prc=$?
tail -25 gpurun_out/pytest_$tag.log
[ $prc -eq 0 ] || [ $prc -eq 1 ] || exit $prc   # 1 = test failures (listed); anything else: stop
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$tag.log 2>&1 || { tail -20 gpurun_out/smoke_$tag.log; exit 1; }
timeout -k 10 500 python bench.py > gpurun_out/bench_$tag.log 2>&1 || { tail -20 gpurun_out/bench_$tag.log; exit 1; }
tail -c 300 gpurun_out/bench_$tag.log
exit $prc
