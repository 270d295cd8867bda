#!/bin/bash
# round 6 job n: the fused QKV + attention in grouped tile order where Wqkv exceeds an XCD's
# 4 MB L2 (C4: 6 MB; A/B build qkv_group.so) against release on the C4 leg, interleaved three
# times; then the C4 GEMM family's HBM traffic (FETCH_SIZE / WRITE_SIZE passes) of both.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6_n
mkdir -p $O
export PYTHONUNBUFFERED=1
V=$R/information-retrieval-with-contrastive-learning_amd/irc_amd/lib/variants
for rep in 1 2 3; do
  for v in release qkv_group; do
    if [ $v = release ]; then unset IRC_LIB_PATH; else export IRC_LIB_PATH=$V/$v.so; fi
    timeout -k 10 300 python bench.py --part train_c4 --steps 10 --warmup 3 --no-cpu-baseline \
      > $O/${v}_$rep.log 2>&1 || { tail $O/${v}_$rep.log; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/${v}_$rep.log').read().strip().splitlines()[-1])
print('$v $rep', round(d['value']), 'pairs/s gemm_frac', d['legs']['train_c4']['gemm_frac'])"
  done
done
GEMM='gemm_big_kernel<|gemm_kernel<unsigned short|gemm_pp_kernel<(true|false), (true|false), [a-z ]+, [0-6], (false|0)(, false)?>|qkv_attn_kernel'
export TMPDIR=/tmp
for v in release qkv_group; do
  if [ $v = release ]; then unset IRC_LIB_PATH; else export IRC_LIB_PATH=$V/$v.so; fi
  cd /tmp || exit 1
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 300 rocprofv3 --pmc $c --output-format csv -d $O/pmc_${v}_$c -o run -- \
      python3 $R/bench.py --part train_c4 --steps 3 --warmup 1 --no-cpu-baseline \
      > $O/pmc_${v}_$c.log 2>&1 || { echo "pass $v $c failed"; tail $O/pmc_${v}_$c.log; exit 1; }
  done
  cd $R || exit 1
  python3 tools/pmc_summary.py $O/pmc_${v}_FETCH_SIZE $O/pmc_${v}_WRITE_SIZE "$GEMM" \
    gemm_bf16_c4_$v --out $O \
    --note "all bf16 GEMM dispatches of bench.py --part train_c4 (BERT-large frozen fwd + BiLSTM head), $v" \
    || exit 1
  python3 -c "
import json; d=json.load(open('$O/pmc_gemm_bf16_c4_$v.json')); print('$v', round(d['hbm_bytes_per_launch']/1e6,1), 'MB per launch')"
done
rm -rf $O/pmc_*_FETCH_SIZE $O/pmc_*_WRITE_SIZE
