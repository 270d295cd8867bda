# Round 4 job c: full GPU suite + smoke, the default bench line, and kernel-trace
# summaries of the training and retrieval parts (profiles/r04_*).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
T=${TAG:-c}
mkdir -p gpurun_out/r4$T
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r4$T/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/r4$T/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r4$T/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4$T/smoke.log 2>&1 || { tail -20 gpurun_out/r4$T/smoke.log; exit 1; }
tail -3 gpurun_out/r4$T/smoke.log
timeout -k 10 600 python bench.py > gpurun_out/r4$T/bench.log 2>&1 || { tail -20 gpurun_out/r4$T/bench.log; exit 1; }
cp gpurun_out/bench_detail.json gpurun_out/r4$T/bench_detail.json 2>/dev/null
grep '^{' gpurun_out/r4$T/bench.log | tail -1 | cut -c1-3000
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r4$T/prof_train -o run -- \
  python3 $GRAFT_REPO_ROOT/bench.py --part train --steps 20 --warmup 5 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/r4$T/prof_train.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r4$T/prof_scan -o run -- \
  python3 $GRAFT_REPO_ROOT/bench.py --part scan --steps 20 --warmup 5 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/r4$T/prof_scan.log 2>&1 || exit 1
cd "$GRAFT_REPO_ROOT"
for p in train scan; do
  python3 tools/prof_summary.py gpurun_out/r4$T/prof_$p > gpurun_out/r4$T/${p}_kernels.txt && head -14 gpurun_out/r4$T/${p}_kernels.txt
  python3 tools/prof_summary.py gpurun_out/r4$T/prof_$p --by-grid > gpurun_out/r4$T/${p}_kernels_grid.txt
  find gpurun_out/r4$T/prof_$p -name "*.db" -delete
done
exit 0
