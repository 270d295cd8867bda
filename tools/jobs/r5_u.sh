#!/bin/bash
# round 5 job u: the frozen encoder split into a whole-wave chunk + a tail chunk on a side
# stream (L = 65..80 batches): parity, step time by padded L (split on / off), main.py
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -q --timeout 200 --timeout-method thread \
  tests/test_bert_split_gpu.py tests/test_qkv_attn_gpu.py tests/test_model_gpu.py tests/test_main_gpu.py \
  tests/test_fp8_encoder_gpu.py > gpurun_out/r5_u_pytest.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/r5_u_pytest.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/e2e_probe.py --steps 30 --by-len --lens 64,65,66,68 > gpurun_out/r5_u_probe_on.log 2>&1 || exit $?
grep -E "ms/step" gpurun_out/r5_u_probe_on.log | grep real | sed 's/^/split on  /'
IRC_BERT_SPLIT=0 timeout -k 10 400 python -u tools/e2e_probe.py --steps 30 --by-len --lens 64,65,66,68 > gpurun_out/r5_u_probe_off.log 2>&1 || exit $?
grep -E "ms/step" gpurun_out/r5_u_probe_off.log | grep real | sed 's/^/split off /'
timeout -k 10 400 python -u tools/e2e_train.py --steps 80 > gpurun_out/r5_u_e2e.log 2>&1 || exit $?
grep -E "end-to-end" gpurun_out/r5_u_e2e.log
timeout -k 10 300 python -u tools/step_events.py --steps 30 --L 65 > gpurun_out/r5_u_events65.log 2>&1 || exit $?
grep -A6 "step" gpurun_out/r5_u_events65.log
