# Round-2 closing run on a fresh box: gpu tests, smoke, bench, kernel-trace summary,
# then the LTOP query-bound knob at Q = 128 / 256 on the retrieval legs.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
timeout -k 10 400 python bench.py > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
tail -c 400 gpurun_out/bench.log
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run -- \
  python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/bench_prof.log 2>&1 || exit 1
cd "$GRAFT_REPO_ROOT"
for mq in 128 256; do
  IRC_SCAN_LTOP_MAXQ=$mq timeout -k 10 300 python bench.py --part scan --no-cpu-baseline > gpurun_out/scan_ltop$mq.log 2>&1 || exit 1
done
exit 0
