#!/bin/bash
# round 5 job z: half as many split-K blocks (diagnostic build splithalf) against release:
# the heads weight-gradient GEMMs alone (dw_bench) and the C2 train leg, interleaved
set -o pipefail
mkdir -p gpurun_out
V=$GRAFT_REPO_ROOT/information-retrieval-with-contrastive-learning_amd/irc_amd/lib/variants/splithalf.so
for i in 1 2 3; do
  timeout -k 10 200 python -u tools/dw_bench.py > gpurun_out/r5_z_big_$i.log 2>&1 || exit $?
  echo "rel   $(grep " us " gpurun_out/r5_z_big_$i.log)"
  IRC_LIB_PATH=$V timeout -k 10 200 python -u tools/dw_bench.py > gpurun_out/r5_z_pp_$i.log 2>&1 || exit $?
  echo "half  $(grep " us " gpurun_out/r5_z_pp_$i.log)"
done
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --part train --no-cpu-baseline > gpurun_out/r5_z_trainbig_$i.log 2>&1 || exit $?
  echo "rel   $(tail -1 gpurun_out/r5_z_trainbig_$i.log | cut -c95-175)"
  IRC_LIB_PATH=$V timeout -k 10 300 python bench.py --part train --no-cpu-baseline > gpurun_out/r5_z_trainpp_$i.log 2>&1 || exit $?
  echo "half  $(tail -1 gpurun_out/r5_z_trainpp_$i.log | cut -c95-175)"
done
