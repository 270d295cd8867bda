#!/bin/bash
# round 5 job f: cluster-LSTM hand-off forms bit identity; e2e step time by padded L
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread \
  tests/test_lstm_coop_variants_gpu.py > gpurun_out/r5_f_pytest.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/r5_f_pytest.log | tail -10
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u tools/e2e_probe.py --steps 30 --by-len > gpurun_out/r5_f_probe.log 2>&1
rc=$?
grep -E "ms/step|Error|error" gpurun_out/r5_f_probe.log | tail -30
exit $rc
