cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAIL" gpurun_out/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 200 python tools/host_time.py --steps 40 2>&1 | grep -E "steps|alone|events" || exit 1
timeout -k 10 400 python bench.py --part train --no-cpu-baseline > gpurun_out/bench_train.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --part bert --no-cpu-baseline > gpurun_out/bench_bert.log 2>&1 || exit 1
tail -c 300 gpurun_out/bench_train.log; echo; tail -c 300 gpurun_out/bench_bert.log
