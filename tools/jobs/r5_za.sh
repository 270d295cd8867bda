#!/bin/bash
# round 5 job za: split-K cap on the LSTM head's dW GEMMs (irc_gemm_ex max_blocks):
# GEMM + head tests, then the C2 train leg with the cap (128, the default) and without
# (IRC_WGRAD_BLOCKS=0), interleaved
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gemm_gpu.py tests/test_lstm_mfma_gpu.py > gpurun_out/r5_za_tests.log 2>&1 || exit $?
tail -2 gpurun_out/r5_za_tests.log
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --part train --no-cpu-baseline > gpurun_out/r5_za_cap_$i.log 2>&1 || exit $?
  echo "cap128 $(tail -1 gpurun_out/r5_za_cap_$i.log | cut -c95-175)"
  IRC_WGRAD_BLOCKS=0 timeout -k 10 300 python bench.py --part train --no-cpu-baseline > gpurun_out/r5_za_full_$i.log 2>&1 || exit $?
  echo "full   $(tail -1 gpurun_out/r5_za_full_$i.log | cut -c95-175)"
done
