# Round 4 job z: bf16 staging in the 256 x 256 kernel's epilogue for bf16 outputs without a
# residual (-DIRC_PP_B16_STAGE): bit-for-bit check, FFN1 timing, C2 step (interleaved A/B).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/r4z
mkdir -p $OUT
V=$GRAFT_REPO_ROOT/information-retrieval-with-contrastive-learning_amd/irc_amd/lib/variants/b16.so
timeout -k 10 120 python tools/variant_bitcheck.py --save $OUT/base.pt > $OUT/bit_base.txt 2>&1 || { tail -5 $OUT/bit_base.txt; exit 1; }
IRC_LIB_PATH=$V timeout -k 10 120 python tools/variant_bitcheck.py --check $OUT/base.pt > $OUT/bit_b16.txt 2>&1 || { tail -14 $OUT/bit_b16.txt; exit 1; }
grep -v amdgpu $OUT/bit_b16.txt
rm -f $OUT/base.pt
SH=ffn1+gelu,ffn1+bias
for r in 1 2 3; do
  timeout -k 10 200 python tools/gemm_bench.py --only $SH > $OUT/g_base_$r.txt 2>&1 || exit 1
  IRC_LIB_PATH=$V timeout -k 10 200 python tools/gemm_bench.py --only $SH > $OUT/g_b16_$r.txt 2>&1 || exit 1
done
for f in g_base_1 g_b16_1 g_base_2 g_b16_2 g_base_3 g_b16_3; do echo "== $f"; grep -v amdgpu $OUT/$f.txt; done
for r in 1 2; do
  for m in base b16; do
    if [ $m = b16 ]; then export IRC_LIB_PATH=$V; else unset IRC_LIB_PATH; fi
    timeout -k 10 200 python bench.py --part train --steps 30 --warmup 5 --no-cpu-baseline > $OUT/train_${m}_$r.log 2>&1 || exit 1
    python3 - $OUT/train_${m}_$r.log $m <<'PY'
import json, sys
d = json.loads([x for x in open(sys.argv[1]) if x.startswith('{')][-1])
print("train %s" % sys.argv[2], round(d["value"]), round(d["ms_per_step"], 3))
PY
  done
done
