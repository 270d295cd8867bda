#!/bin/bash
# round 5 job c: re-check the two failures of b, then time the attention kernels
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread \
  tests/test_model_gpu.py tests/test_train_ops_gpu.py tests/test_attention_gpu.py \
  > gpurun_out/r5_c_pytest.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/r5_c_pytest.log | tail -10
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/attn_bench.py > gpurun_out/r5_c_attn_bench.txt 2>&1
rc=$?
cat gpurun_out/r5_c_attn_bench.txt
exit $rc
