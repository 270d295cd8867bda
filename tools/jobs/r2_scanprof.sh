# Kernel trace of the C2 scan at Q in {1,16,64,256}: per-kernel durations by grid.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python tools/scan_bench.py --reps 30 > gpurun_out/scan_bench.log 2>&1 || exit 1
cat gpurun_out/scan_bench.log
cd /tmp
timeout -k 10 180 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/prof_scan -o run -- \
  python3 $GRAFT_REPO_ROOT/tools/scan_bench.py --reps 30 > $GRAFT_REPO_ROOT/gpurun_out/scan_prof.log 2>&1 || exit 1
exit 0
