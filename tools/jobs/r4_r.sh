# Round 4 job r: ping-pong form of the big-tile main loop (-DIRC_BIG_PP): bit-for-bit
# against the 2-slot loop, tests on the variant, GEMM / fused-layer / C2-step A/B.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/r4r
mkdir -p $OUT
V=$GRAFT_REPO_ROOT/information-retrieval-with-contrastive-learning_amd/irc_amd/lib/variants/bigpp.so
timeout -k 10 120 python tools/variant_bitcheck.py --save $OUT/base.pt > $OUT/bit_base.txt 2>&1 || { tail -5 $OUT/bit_base.txt; exit 1; }
IRC_LIB_PATH=$V timeout -k 10 120 python tools/variant_bitcheck.py --check $OUT/base.pt > $OUT/bit_pp.txt 2>&1 || { tail -12 $OUT/bit_pp.txt; exit 1; }
grep -v amdgpu $OUT/bit_pp.txt
rm -f $OUT/base.pt
IRC_LIB_PATH=$V timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py tests/test_qkv_attn_gpu.py tests/test_ln_fold_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/tests_pp.log 2>&1 || { tail -30 $OUT/tests_pp.log; exit 1; }
tail -1 $OUT/tests_pp.log
SH=qkv,attn_out+res,ffn2+res
for r in 1 2; do
  timeout -k 10 200 python tools/gemm_bench.py --only $SH > $OUT/g_base_$r.txt 2>&1 || exit 1
  IRC_LIB_PATH=$V timeout -k 10 200 python tools/gemm_bench.py --only $SH > $OUT/g_pp_$r.txt 2>&1 || exit 1
  timeout -k 10 100 python tools/qkv_attn_bench.py --iters 30 > $OUT/qa_base_$r.txt 2>&1 || exit 1
  IRC_LIB_PATH=$V timeout -k 10 100 python tools/qkv_attn_bench.py --iters 30 > $OUT/qa_pp_$r.txt 2>&1 || exit 1
done
for f in g_base_1 g_pp_1 g_base_2 g_pp_2 qa_base_1 qa_pp_1 qa_base_2 qa_pp_2; do echo "== $f"; grep -v amdgpu $OUT/$f.txt; done
for r in 1 2; do
  for m in base pp; do
    if [ $m = pp ]; then export IRC_LIB_PATH=$V; else unset IRC_LIB_PATH; fi
    timeout -k 10 200 python bench.py --part train --steps 30 --warmup 5 --no-cpu-baseline > $OUT/train_${m}_$r.log 2>&1 || exit 1
    python3 - $OUT/train_${m}_$r.log $m <<'PY'
import json, sys
d = json.loads([x for x in open(sys.argv[1]) if x.startswith('{')][-1])
print("train %s" % sys.argv[2], round(d["value"]), round(d["ms_per_step"], 3), round(d["roofline"]["frac"], 4))
PY
  done
done
