#!/bin/bash
# round 5 job zf: the head's BPTT split-K cap swept (IRC_HEAD_SPLIT_BLOCKS 96 / 128 / 192),
# C2 train leg, interleaved twice
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  for c in 96 128 192; do
    IRC_HEAD_SPLIT_BLOCKS=$c timeout -k 10 300 python bench.py --part train --no-cpu-baseline > gpurun_out/r5_zf_${c}_$i.log 2>&1 || exit $?
    echo "cap $c: $(tail -1 gpurun_out/r5_zf_${c}_$i.log | cut -c95-175)"
  done
done
