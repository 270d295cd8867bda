#!/bin/bash
# round 6 job i: the packed form of the fused QKV + attention (256 // L sequences a tile at
# L in [32, 51] and [65, 85]): its parity tests, then fused against the two-launch form over
# the sequence lengths a batch's joint padding lands on (B = 32768 // L, and the C2 step's
# 504-sequence chunk at L = 65); and the one-call search_many loop (irc_scan_topk_many):
# its tests, the C2 per-batch time at depths 1-4 against the Python loop and the graphs, and
# the C2 retrieval leg twice.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6_i
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_qkv_attn_gpu.py tests/test_scan_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u tools/qkv_attn_bench.py --iters 20 \
  --lens 32,40,44,48,51,56,60,64,65,72,80,85,90,96,100,112 > $O/bench.log 2>&1 \
  || { tail $O/bench.log; exit 1; }
timeout -k 10 120 python -u tools/qkv_attn_bench.py --iters 20 --b 504 --lens 65 >> $O/bench.log 2>&1 \
  || { tail $O/bench.log; exit 1; }
cat $O/bench.log
timeout -k 10 300 python -u tools/scan_depth.py --reps 200 > $O/scan_depth.log 2>&1 \
  || { tail $O/scan_depth.log; exit 1; }
cat $O/scan_depth.log
for rep in 1 2; do
  timeout -k 10 300 python bench.py --part scan_c2 --steps 10 --warmup 3 --no-cpu-baseline \
    > $O/scan_c2_$rep.log 2>&1 || { tail $O/scan_c2_$rep.log; exit 1; }
  grep -o '"retrieval": {"queries_per_s": [0-9.]*' $O/scan_c2_$rep.log
done
