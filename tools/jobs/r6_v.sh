#!/bin/bash
# round 6 job v: the whole-row MFMA attention backward at any L <= 128 (rows past L read as
# zeros and never stored; was the blocked long kernel at L not a multiple of 32): the
# backward and whole-encoder gradient tests, the attention kernels alone, the --model BERT leg.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6_v
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_bert_train_gpu.py tests/test_attention_gpu.py > $O/pytest.log 2>&1 \
  || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python -u tools/attn_bench.py --lens 32,64,65,72,96,100,128 > $O/attn.log 2>&1 \
  || { tail $O/attn.log; exit 1; }
grep "L=" $O/attn.log | cut -c1-130
timeout -k 10 300 python bench.py --part bert --steps 10 --warmup 3 --no-cpu-baseline \
  > $O/bert.log 2>&1 || { tail $O/bert.log; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bert.log').read().strip().splitlines()[-1]); print('bert', round(d['value']), 'pairs/s')"
