# Persistent 256x256 GEMM A/B: gemm tests, GEMM microbench and the C2 train step, both modes.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_gemm.log 2>&1 || { tail -30 gpurun_out/pytest_gemm.log; exit 1; }
tail -2 gpurun_out/pytest_gemm.log
IRC_GEMM_PERSIST=1 timeout -k 10 200 python tools/gemm_bench.py --iters 30 > gpurun_out/gemm_pers_on.txt 2>&1 || exit 1
IRC_GEMM_PERSIST=0 timeout -k 10 200 python tools/gemm_bench.py --iters 30 > gpurun_out/gemm_pers_off.txt 2>&1 || exit 1
paste gpurun_out/gemm_pers_on.txt gpurun_out/gemm_pers_off.txt | cut -c1-170
IRC_GEMM_PERSIST=1 timeout -k 10 300 python bench.py --part train --no-cpu-baseline > gpurun_out/train_on.log 2>&1 || exit 1
IRC_GEMM_PERSIST=0 timeout -k 10 300 python bench.py --part train --no-cpu-baseline > gpurun_out/train_off.log 2>&1 || exit 1
grep -o '"value": [0-9.]*' gpurun_out/train_on.log | head -1
grep -o '"value": [0-9.]*' gpurun_out/train_off.log | head -1
exit 0
