#!/bin/bash
# round 6 job l: the fused QKV + attention with packed tiles where they take fewer waves and
# the encoder's fused ranges (29-36, 44-64, 80-128): parity tests (fused kernel, encoder,
# scan), then the B = 512 sweep of the release selection.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6_l
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_qkv_attn_gpu.py tests/test_model_gpu.py tests/test_scan_gpu.py > $O/pytest.log 2>&1 \
  || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
LENS=16,20,24,28,29,30,32,34,36,40,44,48,52,56,60,62,63,64,65,68,72,76,80,85,88,92,96,100,104,112,120,128
timeout -k 10 400 python -u tools/qkv_attn_bench.py --iters 20 --b 512 --lens $LENS \
  > $O/sweep.log 2>&1 || { tail $O/sweep.log; exit 1; }
grep "H=" $O/sweep.log | awk '{print $2, $3, $4, $5}' | paste - - - -
