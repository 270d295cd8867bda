#!/bin/bash
# round 5 job h: wave-quantisation heuristic fix -- e2e step time by padded L and main.py
# end to end; GEMM tests; which hipBLASLt kernels torch picks on the BERT shapes
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gemm_gpu.py tests/test_qkv_attn_gpu.py > gpurun_out/r5_h_pytest.log 2>&1
rc=$?
tail -3 gpurun_out/r5_h_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u tools/e2e_probe.py --steps 30 --by-len > gpurun_out/r5_h_probe.log 2>&1 || exit $?
grep -E "ms/step" gpurun_out/r5_h_probe.log
timeout -k 10 400 python -u tools/e2e_train.py --steps 80 > gpurun_out/r5_h_e2e.log 2>&1 || exit $?
grep -E "end-to-end" gpurun_out/r5_h_e2e.log
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5_h_prof -o run -- python3 tools/torch_gemm_ref.py > gpurun_out/r5_h_torch.log 2>&1 || exit $?
tail -12 gpurun_out/r5_h_torch.log
f=$(find gpurun_out/r5_h_prof -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && cut -c1-300 "$f" | head -30
exit 0
