#!/bin/bash
# HBM traffic of the bench's dominant kernels: one FETCH_SIZE and one WRITE_SIZE
# rocprofv3 pass per bench part (counters only, no tracing domains), then
# tools/pmc_summary.py -> gpurun_out/pmc/pmc_<tag>.json (copied to profiles/ by hand).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc
mkdir -p $OUT
cd /tmp
for part in ${PMC_PARTS:-scan_c2 train bert train_fp8}; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 300 rocprofv3 --pmc $c --output-format csv -d $OUT/${part}_$c -o run -- \
      python3 $GRAFT_REPO_ROOT/bench.py --part $part --steps 3 --warmup 1 --no-cpu-baseline \
      > $OUT/${part}_$c.log 2>&1 || { echo "pass $part $c failed"; exit 1; }
  done
done
cd "$GRAFT_REPO_ROOT" || exit 1
# bf16-operand GEMMs (the kernels bench.py's "gemm_bf16" timer covers, the fused QKV +
# attention kernel included); names are demangled
GEMM='gemm_big_kernel<|gemm_kernel<unsigned short|gemm_pp_kernel<(true|false), (true|false), [a-z ]+, [0-6], (false|0)(, false)?>|qkv_attn_kernel'
MX='gemm_pp_kernel<(true|false), (true|false), [a-z ]+, [0-6], 2(, false)?>'
summ() { [ -d "$OUT/$1_FETCH_SIZE" ] || return 0; shift; python3 tools/pmc_summary.py "$@"; }
summ train_fp8 $OUT/train_fp8_FETCH_SIZE $OUT/train_fp8_WRITE_SIZE "$MX" gemm_mx --out $OUT \
  --note "all MX-fp8 GEMM dispatches of bench.py --part train_fp8 (BERT-base frozen fwd on MX-fp8 weights)" || exit 1
summ scan_c2 $OUT/scan_c2_FETCH_SIZE $OUT/scan_c2_WRITE_SIZE \
  'gemm_pp_kernel<true, true, float, 7, (false|0)(, false)?>' scan_filter --out $OUT \
  --note "C2 scan filter (100k x 768 bf16 docs, 256 queries), bench.py --part scan_c2" || exit 1
summ train $OUT/train_FETCH_SIZE $OUT/train_WRITE_SIZE "$GEMM" gemm_bf16 --out $OUT \
  --note "all bf16 GEMM dispatches of bench.py --part train (BERT-base frozen fwd + BiLSTM head)" || exit 1
summ train_c4 $OUT/train_c4_FETCH_SIZE $OUT/train_c4_WRITE_SIZE "$GEMM" gemm_bf16_c4 --out $OUT \
  --note "all bf16 GEMM dispatches of bench.py --part train_c4 (BERT-large frozen fwd + BiLSTM head)" || exit 1
summ bert $OUT/bert_FETCH_SIZE $OUT/bert_WRITE_SIZE "$GEMM" gemm_bf16_bert --out $OUT \
  --note "all bf16 GEMM dispatches of bench.py --part bert (trainable BERT-base fwd+bwd)" || exit 1
exit 0
