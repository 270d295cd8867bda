# Round 4 job h: --model BERT GEMM traffic per family: FETCH_SIZE /
# WRITE_SIZE passes of each fwd / dX / dW shape alone (tools/pmc_shapes.py), the bench
# part's dispatches grouped by family (tools/pmc_family.py), and the shapes' times.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/r4h
mkdir -p $OUT
SH="bert_fwd_qkv bert_fwd_o bert_fwd_ffn1 bert_fwd_ffn2 bert_dx_ffn2 bert_dx_ffn1 bert_dx_qkv bert_dW_ffn1 bert_dW_qkv bert_dW_o"
timeout -k 10 200 python tools/gemm_bench.py --only $(echo $SH | tr ' ' ',') > $OUT/times.txt 2>&1 || exit 1
grep -v amdgpu $OUT/times.txt
cd /tmp
for s in $SH; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d $OUT/${s}_$c -o run -- \
      python3 $GRAFT_REPO_ROOT/tools/gemm_bench.py --only $s --iters 5 > $OUT/${s}_$c.log 2>&1 || { echo "pass $s $c failed"; exit 1; }
  done
done
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $c --output-format csv -d $OUT/bench_$c -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --part bert --steps 3 --warmup 1 --no-cpu-baseline > $OUT/bench_$c.log 2>&1 || { echo "bench pass $c failed"; exit 1; }
done
cd "$GRAFT_REPO_ROOT" || exit 1
python3 tools/pmc_shapes.py $OUT $SH --json $OUT/pmc_shapes_bert.json || exit 1
python3 tools/pmc_family.py $OUT/bench_FETCH_SIZE $OUT/bench_WRITE_SIZE --json $OUT/pmc_family_bert.json || exit 1
find $OUT -name "*.csv" -size +2M -delete
