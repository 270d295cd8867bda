#!/bin/bash
# round 5 job q: v_rcp_f32 sigmoid / tanh in the MFMA recurrences:
# parity (coop forms, LSTM, model, train replay), recurrence timing, stamps, train leg
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -q --timeout 200 --timeout-method thread \
  tests/test_lstm_coop_variants_gpu.py tests/test_lstm_mfma_gpu.py tests/test_model_gpu.py \
  tests/test_train_gpu.py tests/test_configs_gpu.py tests/test_main_gpu.py tests/test_predict_gpu.py > gpurun_out/r5_q_pytest.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/r5_q_pytest.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/lstm_coop_bench.py --ab IRC_NONE=0 > gpurun_out/r5_q_coop.log 2>&1 || exit $?
grep round gpurun_out/r5_q_coop.log
V=$GRAFT_REPO_ROOT/information-retrieval-with-contrastive-learning_amd/irc_amd/lib/variants/coopstamps.so
IRC_LIB_PATH=$V timeout -k 10 200 python -u tools/coop_stamps.py > gpurun_out/r5_q_stamps.log 2>&1 || exit $?
grep -v Warn gpurun_out/r5_q_stamps.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --part train --no-cpu-baseline > gpurun_out/r5_q_train_$i.log 2>&1 || exit $?
  echo "train $(tail -1 gpurun_out/r5_q_train_$i.log | cut -c100-200)"
done
timeout -k 10 300 python -u tools/step_events.py --steps 30 > gpurun_out/r5_q_events.log 2>&1 || exit $?
grep -A6 "step" gpurun_out/r5_q_events.log
