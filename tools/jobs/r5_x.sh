#!/bin/bash
# round 5 job x: the cluster forward's hand-off as per-wave payload + flag (R1) against
# the tagged granules (R2): bit-identity, recurrence timing, the train leg A/B; GEMM ties
# routed to the big-tile kernel (FFN1) under the GEMM / model tests
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread \
  tests/test_lstm_coop_variants_gpu.py tests/test_lstm_mfma_gpu.py tests/test_gemm_gpu.py tests/test_model_gpu.py tests/test_configs_gpu.py > gpurun_out/r5_x_pytest.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/r5_x_pytest.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/lstm_coop_bench.py --ab IRC_LSTM_COOP_WAVE_PUBLISH=1,IRC_LSTM_COOP_WAVE_PUBLISH=2 > gpurun_out/r5_x_coop.log 2>&1 || exit $?
grep round gpurun_out/r5_x_coop.log
for i in 1 2; do
  IRC_LSTM_COOP_WAVE_PUBLISH=1 timeout -k 10 300 python bench.py --part train --no-cpu-baseline > gpurun_out/r5_x_train1_$i.log 2>&1 || exit $?
  echo "R2 $(tail -1 gpurun_out/r5_x_train1_$i.log | cut -c95-190)"
  IRC_LSTM_COOP_WAVE_PUBLISH=2 timeout -k 10 300 python bench.py --part train --no-cpu-baseline > gpurun_out/r5_x_train2_$i.log 2>&1 || exit $?
  echo "R1 $(tail -1 gpurun_out/r5_x_train2_$i.log | cut -c95-190)"
done
