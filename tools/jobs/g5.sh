# GPU parity tests + bench after a scan plan change.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_t.log 2>&1 || exit $?
timeout -k 10 400 python bench.py > gpurun_out/bench_t.log 2>&1 || exit $?
exit 0
