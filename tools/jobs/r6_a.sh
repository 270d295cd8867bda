#!/bin/bash
# round 6 job a: where a whole irc_scan_topk call goes, per kernel, on the C3 shard
# (250k x 768 bf16, beyond the Infinity Cache) at Q = 1 / 16 / 64 / 256 and on C2 at Q = 256.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6_a
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 200 python tools/scan_bench.py --n 250000 --reps 30 > $O/scan_bench_c3.log 2>&1 || { tail $O/scan_bench_c3.log; exit 1; }
cat $O/scan_bench_c3.log
export TMPDIR=/tmp
cd /tmp || exit 1
for cfg in "250000 1" "250000 16" "250000 64" "250000 256" "100000 256"; do
  set -- $cfg
  tag=n$1_q$2
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_$tag -o run -- \
    python3 $R/tools/scan_call_prof.py --n $1 --d 768 --q $2 --reps 20 > $O/prof_$tag.log 2>&1 \
    || { tail $O/prof_$tag.log; exit 1; }
done
cd $R || exit 1
for cfg in n250000_q1 n250000_q16 n250000_q64 n250000_q256 n100000_q256; do
  echo "== $cfg"; tail -1 $O/prof_$cfg.log
  python3 tools/prof_summary.py $O/prof_$cfg > $O/kernels_$cfg.txt && head -8 $O/kernels_$cfg.txt
done
