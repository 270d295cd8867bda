#!/bin/bash
# round 6 job j: the fused QKV + attention with packed tiles only at L in [29, 32] (one
# round of items per head): parity tests, and fused against the two-launch form on a fine
# L grid around the crossovers (host ranges ops.QKV_ATTN_FUSED_L); the C2 retrieval leg at
# depth 4 on the one-call loop.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6_j
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_qkv_attn_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 400 python -u tools/qkv_attn_bench.py --iters 20 \
  --lens 24,28,29,30,31,32,33,36,58,60,61,62,63,64,94,96,97,98,99,100,104 > $O/bench.log 2>&1 \
  || { tail $O/bench.log; exit 1; }
grep "H=" $O/bench.log | awk '{print $2, $4, $5}' | paste - - - -
for rep in 1 2; do
  timeout -k 10 300 python bench.py --part scan_c2 --steps 10 --warmup 3 --no-cpu-baseline \
    > $O/scan_c2_$rep.log 2>&1 || { tail $O/scan_c2_$rep.log; exit 1; }
  grep -o '"retrieval": {"queries_per_s": [0-9.]*' $O/scan_c2_$rep.log
done
