#!/bin/bash
# round 5 job v: the head input projection split (whole-wave rows + tail rows on a side stream)
# on top of the encoder split: parity, step time by padded L (head split on / off), main.py
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -q --timeout 200 --timeout-method thread \
  tests/test_bert_split_gpu.py tests/test_model_gpu.py tests/test_main_gpu.py tests/test_train_gpu.py tests/test_lstm_mfma_gpu.py \
  > gpurun_out/r5_v_pytest.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/r5_v_pytest.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/e2e_probe.py --steps 30 --by-len --lens 64,65,66,68 > gpurun_out/r5_v_probe_on.log 2>&1 || exit $?
grep -E "ms/step" gpurun_out/r5_v_probe_on.log | grep real | sed 's/^/split on  /'
IRC_HEAD_SPLIT=0 timeout -k 10 400 python -u tools/e2e_probe.py --steps 30 --by-len --lens 64,65,66,68 > gpurun_out/r5_v_probe_off.log 2>&1 || exit $?
grep -E "ms/step" gpurun_out/r5_v_probe_off.log | grep real | sed 's/^/split off /'
timeout -k 10 400 python -u tools/e2e_train.py --steps 80 > gpurun_out/r5_v_e2e.log 2>&1 || exit $?
grep -E "end-to-end" gpurun_out/r5_v_e2e.log
timeout -k 10 300 python -u tools/step_events.py --steps 30 --L 65 > gpurun_out/r5_v_events65.log 2>&1 || exit $?
grep -A6 "step" gpurun_out/r5_v_events65.log
