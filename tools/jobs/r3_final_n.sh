# Round-3 closing run at HEAD: full -m gpu suite, smoke, bench, then one kernel-trace
# summary per bench part (train, train_fp8, scan) under rocprofv3 --kernel-trace --stats.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
tag=${1:-n}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rfE --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_$tag.log 2>&1
prc=$?
tail -4 gpurun_out/pytest_$tag.log
[ $prc -eq 0 ] || [ $prc -eq 1 ] || exit $prc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$tag.log 2>&1 || { tail -20 gpurun_out/smoke_$tag.log; exit 1; }
timeout -k 10 500 python bench.py > gpurun_out/bench_$tag.log 2>&1 || { tail -20 gpurun_out/bench_$tag.log; exit 1; }
tail -c 300 gpurun_out/bench_$tag.log
cd /tmp
for part in train train_fp8 scan; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_$part -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --part $part --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof_$part.log 2>&1 || exit 1
done
exit $prc
