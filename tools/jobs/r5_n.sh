#!/bin/bash
# round 5 job n: 64-sequence forward clusters of the LSTM recurrence (half the CUs):
# bit-identity tests, recurrence timing 32 vs 64, the C2 train leg A/B, step timeline
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread \
  tests/test_lstm_coop_variants_gpu.py tests/test_lstm_mfma_gpu.py tests/test_model_gpu.py > gpurun_out/r5_n_pytest.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/r5_n_pytest.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/lstm_coop_bench.py --ab BG=32,BG=64 > gpurun_out/r5_n_coop.log 2>&1 || exit $?
grep round gpurun_out/r5_n_coop.log
for i in 1 2; do
  IRC_LSTM_COOP_BG=32 timeout -k 10 300 python bench.py --part train --no-cpu-baseline > gpurun_out/r5_n_train32_$i.log 2>&1 || exit $?
  echo "BG32 $(tail -1 gpurun_out/r5_n_train32_$i.log | cut -c1-200)"
  IRC_LSTM_COOP_BG=64 timeout -k 10 300 python bench.py --part train --no-cpu-baseline > gpurun_out/r5_n_train64_$i.log 2>&1 || exit $?
  echo "BG64 $(tail -1 gpurun_out/r5_n_train64_$i.log | cut -c1-200)"
done
IRC_LSTM_COOP_BG=32 timeout -k 10 300 python -u tools/step_events.py --steps 30 > gpurun_out/r5_n_events32.log 2>&1 || exit $?
IRC_LSTM_COOP_BG=64 timeout -k 10 300 python -u tools/step_events.py --steps 30 > gpurun_out/r5_n_events64.log 2>&1 || exit $?
cat gpurun_out/r5_n_events32.log gpurun_out/r5_n_events64.log | grep -v Warn
