#!/bin/bash
# round 5 job y: GEMM ties (FFN1: 4 waves of 256x384 vs 6 of 256x256) to the big-tile
# kernel (release) against the round-4 rule (ties to 256x256, diagnostic build tiespp):
# FFN1 alone and the C2 train leg, interleaved
set -o pipefail
mkdir -p gpurun_out
V=$GRAFT_REPO_ROOT/information-retrieval-with-contrastive-learning_amd/irc_amd/lib/variants/tiespp.so
for i in 1 2 3; do
  timeout -k 10 200 python -u tools/gemm_bench.py --only ffn1+gelu --iters 30 > gpurun_out/r5_y_big_$i.log 2>&1 || exit $?
  echo "big   $(grep epi gpurun_out/r5_y_big_$i.log)"
  IRC_LIB_PATH=$V timeout -k 10 200 python -u tools/gemm_bench.py --only ffn1+gelu --iters 30 > gpurun_out/r5_y_pp_$i.log 2>&1 || exit $?
  echo "pp    $(grep epi gpurun_out/r5_y_pp_$i.log)"
done
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --part train --no-cpu-baseline > gpurun_out/r5_y_trainbig_$i.log 2>&1 || exit $?
  echo "big   $(tail -1 gpurun_out/r5_y_trainbig_$i.log | cut -c95-175)"
  IRC_LIB_PATH=$V timeout -k 10 300 python bench.py --part train --no-cpu-baseline > gpurun_out/r5_y_trainpp_$i.log 2>&1 || exit $?
  echo "pp    $(tail -1 gpurun_out/r5_y_trainpp_$i.log | cut -c95-175)"
done
