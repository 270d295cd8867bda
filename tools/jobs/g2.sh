cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python tools/gemm_bench.py --iters 30 > gpurun_out/gemm_bench_s.log 2>&1 || exit $?
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_s.log 2>&1 || exit $?
timeout -k 10 400 python bench.py > gpurun_out/bench_s.log 2>&1 || exit $?
exit 0
