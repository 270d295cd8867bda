# dense_kth window from group maxima: scan parity tests + scan sweep; then the C4 leg's
# own PMC traffic passes (FETCH_SIZE / WRITE_SIZE).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_scan_gpu.py tests/test_scan_fp8_gpu.py tests/test_configs_gpu.py tests/test_predict_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/grp_tests.log 2>&1 || { tail -30 gpurun_out/grp_tests.log; exit 1; }
tail -2 gpurun_out/grp_tests.log
timeout -k 10 400 python bench.py --part scan_c3 --no-cpu-baseline > gpurun_out/grp_scan.log 2>&1 || { tail -20 gpurun_out/grp_scan.log; exit 1; }
python tools/sweep_print.py gpurun_out/grp_scan.log
PMC_PARTS=train_c4 timeout -k 10 700 bash tools/pmc_traffic.sh > gpurun_out/pmc_c4.log 2>&1 || { tail -20 gpurun_out/pmc_c4.log; exit 1; }
cat gpurun_out/pmc/pmc_gemm_bf16_c4.json
