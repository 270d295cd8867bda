#!/bin/bash
# round 5 job g: which hipBLASLt kernels (macro tiles) torch.matmul picks on the BERT shapes
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5_g_prof -o run -- python3 tools/torch_gemm_ref.py > gpurun_out/r5_g_torch.log 2>&1
rc=$?
tail -20 gpurun_out/r5_g_torch.log
f=$(find gpurun_out/r5_g_prof -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && cut -c1-400 "$f" | head -40
exit $rc
