#!/bin/bash
# round 6 job h: grouped GEMM tile order (IRC_GEMM_GROUP_M = 4 / 8 builds) against row-major
# on the C2 and C4 training legs, interleaved twice, then the C4 leg's GEMM HBM traffic under
# the 8-row grouping; and the --model BERT weight-gradient bucket / split-K cap sweep.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6_h
mkdir -p $O
export PYTHONUNBUFFERED=1
V=$R/information-retrieval-with-contrastive-learning_amd/irc_amd/lib/variants
# the attention backward's paired 4-byte stores: the whole-encoder gradient and attention tests
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_bert_train_gpu.py tests/test_attention_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
  for v in release group8 group4; do
    if [ $v = release ]; then unset IRC_LIB_PATH; else export IRC_LIB_PATH=$V/$v.so; fi
    for part in train train_c4; do
      timeout -k 10 300 python bench.py --part $part --steps 10 --warmup 3 --no-cpu-baseline \
        > $O/${v}_${part}_$rep.log 2>&1 || { tail $O/${v}_${part}_$rep.log; exit 1; }
      python3 -c "
import json; d=json.loads(open('$O/${v}_${part}_$rep.log').read().strip().splitlines()[-1])
print('$v $part $rep', round(d['value']), 'pairs/s', d['legs'].get('$part', {}).get('gemm_frac'))"
    done
  done
done
unset IRC_LIB_PATH
export IRC_LIB_PATH=$V/group8.so
cd /tmp || exit 1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $c --output-format csv -d $O/c4g8_$c -o run -- \
    python3 $R/bench.py --part train_c4 --steps 3 --warmup 1 --no-cpu-baseline > $O/c4g8_$c.log 2>&1 || { echo "pass $c failed"; exit 1; }
done
cd $R || exit 1
unset IRC_LIB_PATH
GEMM='gemm_big_kernel<|gemm_kernel<unsigned short|gemm_pp_kernel<(true|false), (true|false), [a-z ]+, [0-6], (false|0)(, false)?>|qkv_attn_kernel'
python3 tools/pmc_summary.py $O/c4g8_FETCH_SIZE $O/c4g8_WRITE_SIZE "$GEMM" gemm_bf16_c4_group8 --out $O --note "C4 GEMMs, 8-row grouped tiles" || exit 1
timeout -k 10 500 python tools/bert_wgrad_ab.py --steps 10 --reps 2 --bucket 2 4 6 --cap 64 128 > $O/wgrad_sweep.log 2>&1 || { tail $O/wgrad_sweep.log; exit 1; }
grep rep $O/wgrad_sweep.log
