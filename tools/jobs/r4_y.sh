# Round 4 job y: the MX LayerNorm on the 4-rows kernel: fp8 encoder tests and the C5 leg.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/r4y
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_fp8_encoder_gpu.py tests/test_encoder_gpu.py -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for r in 1 2; do
  for m in 1 4; do
    IRC_LN_ROWS=$m timeout -k 10 300 python bench.py --part train_fp8 --steps 30 --warmup 5 --no-cpu-baseline > $OUT/fp8_${m}_$r.log 2>&1 || exit 1
    python3 - $OUT/fp8_${m}_$r.log $m <<'PY'
import json, sys
d = json.loads([x for x in open(sys.argv[1]) if x.startswith('{')][-1])
t = d.get("train_fp8", d)
print("train_fp8 ln_rows=%s" % sys.argv[2], round(d["value"]), round(d["ms_per_step"], 3))
PY
  done
done
