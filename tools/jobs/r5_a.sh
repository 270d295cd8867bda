#!/bin/bash
# round 5 job a: any-L attention (forward streamed, backward block-looped) parity
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_attention_gpu.py tests/test_bert_train_gpu.py tests/test_model_gpu.py \
  tests/test_fp8_encoder_gpu.py::test_attention_mx_equals_quantised_attention \
  tests/test_main_gpu.py::test_main_train_long_sentences \
  > gpurun_out/r5_a_pytest.log 2>&1
rc=$?
tail -30 gpurun_out/r5_a_pytest.log
exit $rc
