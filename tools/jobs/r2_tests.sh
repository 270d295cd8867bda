# Selected GPU test files (arguments), one pytest process, per-test timeout.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest "$@" -m gpu -v -s --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_sel.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed|rel |err |C2 step|loss " gpurun_out/pytest_sel.log | tail -60
exit $rc
