#!/bin/bash
# round 5 job zg: grid cap of the ping-pong GEMM (irc_gemm_ex max_blocks as a static
# persistent tile loop) -- GEMM tests, then the C2 train leg with the LSTM head's input
# projection capped at 0 (off) / 128 / 192 workgroups, interleaved
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_gemm_gpu.py tests/test_lstm_mfma_gpu.py > gpurun_out/r5_zg_tests.log 2>&1 || { tail -30 gpurun_out/r5_zg_tests.log; exit 1; }
tail -1 gpurun_out/r5_zg_tests.log
for i in 1 2 3; do
  for c in 0 128 192; do
    IRC_HEAD_PROJ_BLOCKS=$c timeout -k 10 300 python bench.py --part train --no-cpu-baseline > gpurun_out/r5_zg_${c}_$i.log 2>&1 || exit $?
    echo "proj $c: $(tail -1 gpurun_out/r5_zg_${c}_$i.log | cut -c95-175)"
  done
done
