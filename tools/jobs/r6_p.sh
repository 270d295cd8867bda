#!/bin/bash
# round 6 job p: attention skips the key blocks past a sequence's last visible key
# (visible_key_blocks, exact): parity tests of every attention consumer, then release
# against the no-skip A/B build on the C2 and C5 legs and the L = 65 QKV + attention
# layer (interleaved twice), and main.py end to end once each.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6_p
mkdir -p $O
export PYTHONUNBUFFERED=1
V=$R/information-retrieval-with-contrastive-learning_amd/irc_amd/lib/variants
timeout -k 10 700 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_attention_gpu.py tests/test_qkv_attn_gpu.py tests/test_model_gpu.py \
  tests/test_fp8_encoder_gpu.py tests/test_bert_train_gpu.py > $O/pytest.log 2>&1 \
  || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
  for v in release noskip; do
    if [ $v = release ]; then unset IRC_LIB_PATH; else export IRC_LIB_PATH=$V/$v.so; fi
    for part in train train_fp8; do
      timeout -k 10 300 python bench.py --part $part --steps 10 --warmup 3 --no-cpu-baseline \
        > $O/${v}_${part}_$rep.log 2>&1 || { tail $O/${v}_${part}_$rep.log; exit 1; }
      python3 -c "
import json; d=json.loads(open('$O/${v}_${part}_$rep.log').read().strip().splitlines()[-1])
print('$v $part $rep', round(d['value']), 'pairs/s')"
    done
    timeout -k 10 120 python -u tools/qkv_attn_bench.py --iters 20 --b 504 --lens 65 \
      > $O/${v}_qkv65_$rep.log 2>&1 || { tail $O/${v}_qkv65_$rep.log; exit 1; }
    echo "$v qkv65: $(grep H= $O/${v}_qkv65_$rep.log | awk '{print $4, $5}' | tr '\n' ' ')"
  done
done
for v in release noskip; do
  if [ $v = release ]; then unset IRC_LIB_PATH; else export IRC_LIB_PATH=$V/$v.so; fi
  timeout -k 10 400 python -u tools/e2e_train.py --steps 80 > $O/${v}_e2e.log 2>&1 \
    || { tail $O/${v}_e2e.log; exit 1; }
  echo "$v $(grep end-to-end $O/${v}_e2e.log)"
done
