#!/bin/bash
# round 5 job k: A/B of the GEMM wave-remainder split (IRC_GEMM_REMAINDER) on the step
# time by padded L, with the LayerNorm's __restrict__ restored
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for r in 1 0 1 0; do
  echo "IRC_GEMM_REMAINDER=$r"
  IRC_GEMM_REMAINDER=$r timeout -k 10 400 python -u tools/e2e_probe.py --steps 30 --by-len --lens 62,64,65,67 > gpurun_out/r5_k_probe_$r.log 2>&1 || exit $?
  grep -E "ms/step" gpurun_out/r5_k_probe_$r.log | grep real
done
timeout -k 10 300 python -u bench.py --part train --no-cpu-baseline > gpurun_out/r5_k_bench_train.log 2>&1 || exit $?
tail -1 gpurun_out/r5_k_bench_train.log | cut -c1-200
