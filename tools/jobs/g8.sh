# Kernel trace of the retrieval part (dense C2/C4/C5 legs + sparse TF-IDF leg).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
cd /tmp || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_u_scan" -o run -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --part scan --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/prof_u_scan.log" 2>&1 || exit $?
exit 0
