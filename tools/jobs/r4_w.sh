# Round 4 job w: LayerNorm with 4 rows per half-wave (IRC_LN_ROWS=4): bit-for-bit against
# the one-row kernel, the kernel time, and the C2 step (interleaved); the vectorised
# embedding gather + LN and the encoder / model / config tests.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/r4w
mkdir -p $OUT
timeout -k 10 120 python tools/variant_bitcheck.py --save $OUT/base.pt > $OUT/bit_base.txt 2>&1 || { tail -5 $OUT/bit_base.txt; exit 1; }
IRC_LN_ROWS=4 timeout -k 10 120 python tools/variant_bitcheck.py --check $OUT/base.pt > $OUT/bit_ln4.txt 2>&1 || { tail -12 $OUT/bit_ln4.txt; exit 1; }
grep -v amdgpu $OUT/bit_ln4.txt
rm -f $OUT/base.pt
for r in 1 2 3; do
  timeout -k 10 60 python tools/ln_bench.py >> $OUT/ln.txt 2>&1 || exit 1
  IRC_LN_ROWS=4 timeout -k 10 60 python tools/ln_bench.py >> $OUT/ln.txt 2>&1 || exit 1
done
grep -v amdgpu $OUT/ln.txt
timeout -k 10 300 python -u -m pytest tests/test_encoder_gpu.py tests/test_model_gpu.py tests/test_configs_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for r in 1 2; do
  for m in 1 4; do
    IRC_LN_ROWS=$m timeout -k 10 200 python bench.py --part train --steps 30 --warmup 5 --no-cpu-baseline > $OUT/train_${m}_$r.log 2>&1 || exit 1
    python3 - $OUT/train_${m}_$r.log $m <<'PY'
import json, sys
d = json.loads([x for x in open(sys.argv[1]) if x.startswith('{')][-1])
print("train ln_rows=%s" % sys.argv[2], round(d["value"]), round(d["ms_per_step"], 3))
PY
  done
done
