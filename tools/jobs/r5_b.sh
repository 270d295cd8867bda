#!/bin/bash
# round 5 job b: any-L attention + SGD / activations parity
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest -v --timeout 300 --timeout-method thread \
  tests/test_attention_gpu.py tests/test_bert_train_gpu.py tests/test_model_gpu.py \
  tests/test_fp8_encoder_gpu.py::test_attention_mx_equals_quantised_attention \
  tests/test_main_gpu.py::test_main_train_long_sentences tests/test_train_gpu.py \
  tests/test_train_ops_gpu.py \
  > gpurun_out/r5_b_pytest.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/r5_b_pytest.log | tail -30
exit $rc
