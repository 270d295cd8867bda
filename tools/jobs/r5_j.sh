#!/bin/bash
# round 5 job j: fused QKV+attention up to L = 128, GEMM wave remainder -- parity;
# fused vs two-launch by L; step time by padded L; main.py end to end; train leg
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread \
  tests/test_gemm_gpu.py tests/test_qkv_attn_gpu.py tests/test_encoder_gpu.py \
  tests/test_configs_gpu.py tests/test_train_gpu.py > gpurun_out/r5_j_pytest.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/r5_j_pytest.log | tail -12
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/qkv_attn_bench.py --lens 40,48,56,60,63,64,65,72,80,96,100,112,120,128 > gpurun_out/r5_j_qkv.log 2>&1 || exit $?
grep -E "us" gpurun_out/r5_j_qkv.log | awk 'NR%4==3 || NR%4==0'
timeout -k 10 500 python -u tools/e2e_probe.py --steps 30 --by-len > gpurun_out/r5_j_probe.log 2>&1 || exit $?
grep -E "ms/step" gpurun_out/r5_j_probe.log
timeout -k 10 400 python -u tools/e2e_train.py --steps 80 > gpurun_out/r5_j_e2e.log 2>&1 || exit $?
grep -E "end-to-end" gpurun_out/r5_j_e2e.log
timeout -k 10 300 python -u bench.py --part train --no-cpu-baseline > gpurun_out/r5_j_bench_train.log 2>&1 || exit $?
tail -1 gpurun_out/r5_j_bench_train.log | cut -c1-200
