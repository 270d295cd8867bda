# Round 4 job p: C5 (MX-fp8 encoder) after the scale-fill fix: tests, the leg, its kernels.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/r4p
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_fp8_encoder_gpu.py tests/test_configs_gpu.py -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 300 python bench.py --part train_fp8 --steps 30 --warmup 5 --no-cpu-baseline > $OUT/fp8.log 2>&1 || exit 1
python3 - $OUT/fp8.log <<'PY'
import json, sys
d = json.loads([x for x in open(sys.argv[1]) if x.startswith('{')][-1])
t = d.get("train_fp8", d)
print("train_fp8", json.dumps(t)[:300])
PY
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_fp8 -o run -- \
  python3 $GRAFT_REPO_ROOT/bench.py --part train_fp8 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/prof_fp8.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && python3 tools/prof_summary.py $OUT/prof_fp8 --by-grid > $OUT/fp8_kernels.txt && head -24 $OUT/fp8_kernels.txt
find $OUT -name "*.db" -delete
