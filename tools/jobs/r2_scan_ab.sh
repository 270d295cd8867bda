# Scan parity tests, then the Q sweep (call and filter times) of the current build.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_scan_gpu.py tests/test_scan_fp8_gpu.py tests/test_configs_gpu.py \
  tests/test_predict_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_scan.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_scan.log; [ $rc -ne 0 ] && { grep -E "Error|assert" gpurun_out/pytest_scan.log | head -20; exit $rc; }
timeout -k 10 120 python tools/scan_bench.py --q 1 16 64 128 256 --reps 50 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 120 python tools/scan_bench.py --q 1 64 256 --reps 30 --fp8 2>&1 | grep -v amdgpu.ids || exit 1
