#!/bin/bash
# round 5 job l: remainder split priced in us (FFN2 only at L = 65..72): parity, step time
# by padded L, main.py end to end; kernel traces of the step at L = 64 and 65
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread \
  tests/test_gemm_gpu.py -k "remainder" > gpurun_out/r5_l_pytest.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/r5_l_pytest.log | tail -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/e2e_probe.py --steps 30 --by-len --lens 62,63,64,65,66,67,68 > gpurun_out/r5_l_probe.log 2>&1 || exit $?
grep -E "ms/step" gpurun_out/r5_l_probe.log | grep real
timeout -k 10 400 python -u tools/e2e_train.py --steps 80 > gpurun_out/r5_l_e2e.log 2>&1 || exit $?
grep -E "end-to-end" gpurun_out/r5_l_e2e.log
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for L in 64 65; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r5_l_prof_$L -o run -- python3 tools/e2e_probe.py --steps 30 --by-len --lens $L > gpurun_out/r5_l_tprobe_$L.log 2>&1 || exit $?
done
python3 tools/trace_top.py gpurun_out/r5_l_prof_64 --top 25
python3 tools/trace_top.py gpurun_out/r5_l_prof_65 --top 25
