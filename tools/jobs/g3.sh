# Round-end evidence: smoke(), then rocprofv3 kernel traces of the full bench and of the
# training part alone (each step under its own time limit; the chain stops at a failure).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_s.log 2>&1 || exit $?
cd /tmp || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_s" -o run -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/prof_s.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_s_train" -o run -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --part train --steps 3 --warmup 1 --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/prof_s_train.log" 2>&1 || exit $?
exit 0
