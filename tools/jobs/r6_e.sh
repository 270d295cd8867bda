#!/bin/bash
# round 6 job e: the interleaved-DMA build (IRC_SCAN_IL=1) against the release build on the
# single-pass scan up to Q = 128 (IRC_SCAN_LTOP_MAXQ=128) and on the sampled tile pipeline,
# C3 and C2 shards, two interleaved repetitions.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6_e
mkdir -p $O
export PYTHONUNBUFFERED=1
V=$R/information-retrieval-with-contrastive-learning_amd/irc_amd/lib/variants
for rep in 1 2; do
  for v in release IL; do
    if [ $v = release ]; then unset IRC_LIB_PATH; else export IRC_LIB_PATH=$V/scan_$v.so; fi
    for n in 250000 100000; do
      echo "== $v ltop128 N=$n ($rep)"
      IRC_SCAN_LTOP_MAXQ=128 timeout -k 10 120 python tools/scan_bench.py --n $n --reps 30 \
        --q 1 16 48 64 96 128 > $O/${v}_ltop_n${n}_$rep.log 2>&1 || { tail $O/${v}_ltop_n${n}_$rep.log; exit 1; }
      grep filter $O/${v}_ltop_n${n}_$rep.log
      echo "== $v sampled N=$n ($rep)"
      IRC_SCAN_LTOP=0 timeout -k 10 120 python tools/scan_bench.py --n $n --reps 30 \
        --q 64 96 128 > $O/${v}_samp_n${n}_$rep.log 2>&1 || { tail $O/${v}_samp_n${n}_$rep.log; exit 1; }
      grep filter $O/${v}_samp_n${n}_$rep.log
    done
  done
done
