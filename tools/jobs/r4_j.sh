# Round 4 job j: XCD remap over the whole grid (batch, split, tile) in gemm_pp_kernel:
# GEMM / trainable-encoder tests, dW shapes new vs old remap (interleaved), their HBM
# traffic, and the --model BERT step with each.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/r4j
mkdir -p $OUT
V=$GRAFT_REPO_ROOT/information-retrieval-with-contrastive-learning_amd/irc_amd/lib/variants/oldremap.so
timeout -k 10 500 python -u -m pytest tests/test_gemm_gpu.py tests/test_bert_train_gpu.py tests/test_train_ops_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
SH=bert_dW_ffn1,bert_dW_qkv,bert_dW_o,dW_ih^T,dW_hh^T
for r in 1 2; do
  timeout -k 10 200 python tools/gemm_bench.py --only $SH > $OUT/dw_new_$r.txt 2>&1 || exit 1
  IRC_LIB_PATH=$V timeout -k 10 200 python tools/gemm_bench.py --only $SH > $OUT/dw_old_$r.txt 2>&1 || exit 1
done
for f in dw_new_1 dw_old_1 dw_new_2 dw_old_2; do echo "== $f"; grep -v amdgpu $OUT/$f.txt; done
for r in 1 2; do
  for m in new old; do
    if [ $m = old ]; then export IRC_LIB_PATH=$V; else unset IRC_LIB_PATH; fi
    timeout -k 10 300 python bench.py --part bert --steps 10 --warmup 3 --no-cpu-baseline > $OUT/bert_${m}_$r.log 2>&1 || exit 1
    python3 - $OUT/bert_${m}_$r.log $m <<'PY'
import json, sys
d = json.loads([x for x in open(sys.argv[1]) if x.startswith('{')][-1])
b = d.get("train_bert", d)
print("bert remap=%s" % sys.argv[2], round(b["value"]) if "value" in b else b.get("pairs_per_s"), round(b["ms_per_step"], 3), b.get("roofline", {}).get("frac"))
PY
  done
done
unset IRC_LIB_PATH
cd /tmp
for s in bert_dW_ffn1 bert_dW_qkv bert_dW_o; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d $OUT/${s}_$c -o run -- \
      python3 $GRAFT_REPO_ROOT/tools/gemm_bench.py --only $s --iters 5 > $OUT/${s}_$c.log 2>&1 || { echo "pass $s $c failed"; exit 1; }
  done
done
cd $GRAFT_REPO_ROOT && python3 tools/pmc_shapes.py $OUT bert_dW_ffn1 bert_dW_qkv bert_dW_o --json $OUT/pmc_dw.json
find $OUT -name "*.csv" -size +2M -delete
