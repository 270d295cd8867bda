# Kernel trace of scan_bench (per-kernel durations in each call) for the given Q values.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
cd /tmp
timeout -k 10 180 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/prof_scan -o run -- \
  python3 $GRAFT_REPO_ROOT/tools/scan_bench.py --reps 20 --q "$@" > $GRAFT_REPO_ROOT/gpurun_out/scan_prof.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && python tools/call_timeline.py gpurun_out/prof_scan
