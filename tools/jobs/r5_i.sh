#!/bin/bash
# round 5 job i: slotted fused QKV+attention and the GEMM wave-remainder split -- parity,
# then the step time by padded L, main.py end to end and the bench's train leg
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread \
  tests/test_gemm_gpu.py tests/test_qkv_attn_gpu.py tests/test_encoder_gpu.py \
  tests/test_configs_gpu.py tests/test_train_gpu.py > gpurun_out/r5_i_pytest.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/r5_i_pytest.log | tail -12
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u tools/e2e_probe.py --steps 30 --by-len > gpurun_out/r5_i_probe.log 2>&1 || exit $?
grep -E "ms/step" gpurun_out/r5_i_probe.log
timeout -k 10 400 python -u tools/e2e_train.py --steps 80 > gpurun_out/r5_i_e2e.log 2>&1 || exit $?
grep -E "end-to-end" gpurun_out/r5_i_e2e.log
timeout -k 10 300 python -u bench.py --part train --no-cpu-baseline > gpurun_out/r5_i_bench_train.log 2>&1 || exit $?
tail -1 gpurun_out/r5_i_bench_train.log | cut -c1-200
