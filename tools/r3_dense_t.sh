# select_dense after the one-atomic collect and the vector rank: scan parity tests, phase
# stamps (diagnostic build), then the scan bench part (C2 / C3 Q sweeps).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_scan_gpu.py tests/test_scan_fp8_gpu.py tests/test_configs_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/dense_tests.log 2>&1 || { tail -30 gpurun_out/dense_tests.log; exit 1; }
tail -2 gpurun_out/dense_tests.log
V=$GRAFT_REPO_ROOT/information-retrieval-with-contrastive-learning_amd/irc_amd/lib/variants
IRC_LIB_PATH=$V/stamps.so timeout -k 10 200 python tools/dense_time.py > gpurun_out/dense_time3.txt 2>&1 || { tail -20 gpurun_out/dense_time3.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/dense_time3.txt
timeout -k 10 400 python bench.py --part scan --no-cpu-baseline > gpurun_out/dense_scan.log 2>&1 || { tail -20 gpurun_out/dense_scan.log; exit 1; }
python tools/sweep_print.py gpurun_out/dense_scan.log
