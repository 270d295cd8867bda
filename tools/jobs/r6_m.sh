#!/bin/bash
# round 6 job m: the C2 retrieval leg at 3 and 4 batches in flight on the one-call loop,
# interleaved on one box, with the depth tool beside it.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6_m
mkdir -p $O
export PYTHONUNBUFFERED=1
for rep in 1 2 3; do
  for d in 3 4; do
    timeout -k 10 300 python bench.py --part scan_c2 --steps 10 --warmup 3 --no-cpu-baseline \
      --scan-depth $d > $O/scan_c2_d${d}_$rep.log 2>&1 || { tail $O/scan_c2_d${d}_$rep.log; exit 1; }
    echo "depth $d rep $rep $(grep -o '"retrieval": {"queries_per_s": [0-9.]*' $O/scan_c2_d${d}_$rep.log)"
  done
done
timeout -k 10 300 python -u tools/scan_depth.py --reps 200 > $O/scan_depth.log 2>&1 \
  || { tail $O/scan_depth.log; exit 1; }
grep native $O/scan_depth.log
