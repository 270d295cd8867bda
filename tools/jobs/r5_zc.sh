#!/bin/bash
# round 5 job zc: C2 train leg, interleaved three times: release (split-K cap 128 on the LSTM
# head's dW GEMMs only), the split128 build (every split GEMM capped at 128, as job z's
# diagnostic), and release with the dW cap at 64
set -o pipefail
mkdir -p gpurun_out
V=$GRAFT_REPO_ROOT/information-retrieval-with-contrastive-learning_amd/irc_amd/lib/variants/split128.so
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --part train --no-cpu-baseline > gpurun_out/r5_zc_rel_$i.log 2>&1 || exit $?
  echo "rel      $(tail -1 gpurun_out/r5_zc_rel_$i.log | cut -c95-175)"
  IRC_LIB_PATH=$V timeout -k 10 300 python bench.py --part train --no-cpu-baseline > gpurun_out/r5_zc_all_$i.log 2>&1 || exit $?
  echo "all128   $(tail -1 gpurun_out/r5_zc_all_$i.log | cut -c95-175)"
  IRC_WGRAD_BLOCKS=64 timeout -k 10 300 python bench.py --part train --no-cpu-baseline > gpurun_out/r5_zc_w64_$i.log 2>&1 || exit $?
  echo "wgrad64  $(tail -1 gpurun_out/r5_zc_w64_$i.log | cut -c95-175)"
done
