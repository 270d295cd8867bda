#!/bin/bash
# round 6 job c: where the single-pass (LTOP) filter's time goes on the C3 shard at
# Q = 1 / 16 / 32 / 64: release build against the diagnostic builds (corpus stream only,
# + MFMAs, + k-slice exchange without the list epilogue).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6_c
mkdir -p $O
export PYTHONUNBUFFERED=1
V=$R/information-retrieval-with-contrastive-learning_amd/irc_amd/lib/variants
for rep in 1 2; do
  for v in release IL DMA_ONLY MFMA_ONLY NO_EPI; do
    if [ $v = release ]; then unset IRC_LIB_PATH; else export IRC_LIB_PATH=$V/scan_$v.so; fi
    echo "== $v ($rep)"
    timeout -k 10 120 python tools/scan_bench.py --n 250000 --reps 30 --q 1 16 32 64 \
      > $O/${v}_$rep.log 2>&1 || { tail $O/${v}_$rep.log; exit 1; }
    grep "filter" $O/${v}_$rep.log
  done
done
# the stationary-query tile kernel (sampled threshold) against the GEMM filter at Q >= 128
unset IRC_LIB_PATH
for pp in 1 0; do
  for n in 250000 100000; do
    echo "== IRC_SCAN_PP=$pp N=$n"
    IRC_SCAN_PP=$pp timeout -k 10 120 python tools/scan_bench.py --n $n --reps 30 --q 128 192 256 512 \
      > $O/pp${pp}_n$n.log 2>&1 || { tail $O/pp${pp}_n$n.log; exit 1; }
    grep "filter" $O/pp${pp}_n$n.log
  done
done
# the single-pass (LTOP) tile kernel at Q >= 128
for n in 250000 100000; do
  echo "== IRC_SCAN_PP=0 LTOP_MAXQ=512 N=$n"
  IRC_SCAN_PP=0 IRC_SCAN_LTOP_MAXQ=512 timeout -k 10 120 python tools/scan_bench.py --n $n --reps 30 \
    --q 128 192 256 512 > $O/ltop_n$n.log 2>&1 || { tail $O/ltop_n$n.log; exit 1; }
  grep "filter" $O/ltop_n$n.log
done
# phase stamps (block 0) of the sampled pipeline at Q = 256 on both filters
for pp in 1 0; do
  echo "== stamps IRC_SCAN_PP=$pp"
  IRC_SCAN_PP=$pp IRC_LIB_PATH=$V/scan_STAMPS.so timeout -k 10 120 python tools/scan_stamps.py \
    --n 250000 --q 1 64 256 > $O/stamps_pp$pp.log 2>&1 || { tail $O/stamps_pp$pp.log; exit 1; }
  cat $O/stamps_pp$pp.log
done
