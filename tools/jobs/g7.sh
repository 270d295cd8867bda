# Sparse path change: sparse GPU tests, then the sparse bench leg via the full scan part.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_sparse_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_sparse_u.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --part scan --no-cpu-baseline > gpurun_out/bench_scan_u.log 2>&1 || exit $?
exit 0
