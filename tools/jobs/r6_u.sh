#!/bin/bash
# round 6 job u: the whole-row MFMA attention as one workgroup per (sequence, head) with one
# shared V^T image (was: 4 unrelated waves a workgroup, each with its own copy): parity tests
# of every consumer, then against the previous kernel (attn_old.so) -- attention alone at
# 32k tokens, the C5 leg, main.py end to end -- interleaved.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6_u
mkdir -p $O
export PYTHONUNBUFFERED=1
V=$R/information-retrieval-with-contrastive-learning_amd/irc_amd/lib/variants
timeout -k 10 700 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_attention_gpu.py tests/test_qkv_attn_gpu.py tests/test_model_gpu.py \
  tests/test_fp8_encoder_gpu.py tests/test_bert_train_gpu.py tests/test_bert_split_gpu.py \
  > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
  for v in new old; do
    if [ $v = new ]; then unset IRC_LIB_PATH; else export IRC_LIB_PATH=$V/attn_old.so; fi
    timeout -k 10 200 python -u tools/attn_bench.py --lens 32,64,65,72,96,128 > $O/${v}_attn_$rep.log 2>&1 \
      || { tail $O/${v}_attn_$rep.log; exit 1; }
    echo "== $v $rep"; grep "L=" $O/${v}_attn_$rep.log | cut -c1-80
    timeout -k 10 300 python bench.py --part train_fp8 --steps 10 --warmup 3 --no-cpu-baseline \
      > $O/${v}_fp8_$rep.log 2>&1 || { tail $O/${v}_fp8_$rep.log; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/${v}_fp8_$rep.log').read().strip().splitlines()[-1])
print('$v fp8 $rep', round(d['value']), 'pairs/s')"
  done
done
for v in new old; do
  if [ $v = new ]; then unset IRC_LIB_PATH; else export IRC_LIB_PATH=$V/attn_old.so; fi
  timeout -k 10 400 python -u tools/e2e_train.py --steps 80 > $O/${v}_e2e.log 2>&1 \
    || { tail $O/${v}_e2e.log; exit 1; }
  echo "$v $(grep end-to-end $O/${v}_e2e.log)"
done
