# Round 4 job g: the LayerNorm fold (irc_gemm_ln): parity tests, then the C2 / C4
# training steps with and without the fold, interleaved on one box, and a kernel trace
# of the folded frozen encoder.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r4g
timeout -k 10 500 python -u -m pytest tests/test_ln_fold_gpu.py tests/test_encoder_gpu.py tests/test_model_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r4g/tests.log 2>&1 || { tail -40 gpurun_out/r4g/tests.log; exit 1; }
tail -1 gpurun_out/r4g/tests.log
for r in 1 2; do
  for f in 0 1; do
    IRC_LN_FOLD=$f timeout -k 10 200 python bench.py --part train --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/r4g/train_${f}_$r.log 2>&1 || exit 1
    python3 - gpurun_out/r4g/train_${f}_$r.log $f <<'PY'
import json, sys
d = json.loads([x for x in open(sys.argv[1]) if x.startswith('{')][-1])
print("train fold=%s" % sys.argv[2], round(d["value"]), round(d["ms_per_step"], 3), round(d["roofline"]["frac"], 4))
PY
  done
done
for f in 0 1; do
  IRC_LN_FOLD=$f timeout -k 10 300 python bench.py --part train_c4 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r4g/c4_${f}.log 2>&1 || exit 1
  python3 - gpurun_out/r4g/c4_${f}.log $f <<'PY'
import json, sys
d = json.loads([x for x in open(sys.argv[1]) if x.startswith('{')][-1])
c = d.get("train_c4", d)
print("c4 fold=%s" % sys.argv[2], json.dumps(c)[:300])
PY
done
cd /tmp
for f in 0 1; do
  IRC_LN_FOLD=$f timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r4g/bert_f$f -o run -- \
    python3 $GRAFT_REPO_ROOT/tools/overlap_prof.py --mode bert --steps 20 > $GRAFT_REPO_ROOT/gpurun_out/r4g/bert_f$f.log 2>&1 || exit 1
  (cd $GRAFT_REPO_ROOT && grep "mode" gpurun_out/r4g/bert_f$f.log | tail -1 && python3 tools/prof_summary.py gpurun_out/r4g/bert_f$f --by-grid > gpurun_out/r4g/bert_f${f}_kernels.txt && head -16 gpurun_out/r4g/bert_f${f}_kernels.txt)
  find $GRAFT_REPO_ROOT/gpurun_out/r4g/bert_f$f -name "*.db" -delete
done
