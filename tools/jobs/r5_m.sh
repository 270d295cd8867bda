#!/bin/bash
# round 5 job m: wave tail of the big-tile GEMM (K pieces in the same launch): parity,
# per-shape timing on/off, step time by padded L, main.py end to end
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread \
  tests/test_gemm_gpu.py > gpurun_out/r5_m_pytest.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/r5_m_pytest.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/tail_bench.py > gpurun_out/r5_m_tail.log 2>&1 || exit $?
cat gpurun_out/r5_m_tail.log | grep "L="
timeout -k 10 400 python -u tools/e2e_probe.py --steps 30 --by-len --lens 62,64,65,66,68 > gpurun_out/r5_m_probe.log 2>&1 || exit $?
grep -E "ms/step" gpurun_out/r5_m_probe.log | grep real
timeout -k 10 400 python -u tools/e2e_train.py --steps 80 > gpurun_out/r5_m_e2e.log 2>&1 || exit $?
grep -E "end-to-end" gpurun_out/r5_m_e2e.log
timeout -k 10 300 python -u tools/step_events.py --steps 30 --L 64 > gpurun_out/r5_m_events64.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/step_events.py --steps 30 --L 65 > gpurun_out/r5_m_events65.log 2>&1 || exit $?
grep -A8 "step" gpurun_out/r5_m_events64.log gpurun_out/r5_m_events65.log
