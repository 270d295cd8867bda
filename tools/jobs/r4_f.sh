# Round 4 job f: the big-tile kernel's 16x16x32 form: exactness tests, interleaved GEMM A/B
# on the BERT shapes, and the C2 training step with each form (same box).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r4f
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "mf16 or big_tile or gelu" > gpurun_out/r4f/tests.log 2>&1 || { tail -30 gpurun_out/r4f/tests.log; exit 1; }
tail -1 gpurun_out/r4f/tests.log
timeout -k 10 300 python tools/gemm_bench.py --only qkv,attn_out+res,ffn2+res,ffn1+gelu --mf16 ab > gpurun_out/r4f/gemm_ab.txt 2>&1 || exit 1
grep -v amdgpu gpurun_out/r4f/gemm_ab.txt
for r in 1 2; do
  for m in 0 1; do
    IRC_BIG_MF16=$m timeout -k 10 200 python bench.py --part train --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/r4f/train_${m}_$r.log 2>&1 || exit 1
    python3 - gpurun_out/r4f/train_${m}_$r.log $m <<'PY'
import json, sys
d = json.loads([x for x in open(sys.argv[1]) if x.startswith('{')][-1])
print("train mf16=%s" % sys.argv[2], round(d["value"]), round(d["ms_per_step"], 3), round(d["roofline"]["frac"], 4))
PY
  done
done
cd /tmp
for mode in bert overlap heads; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r4f/ov_$mode -o run -- \
    python3 $GRAFT_REPO_ROOT/tools/overlap_prof.py --mode $mode --steps 20 > $GRAFT_REPO_ROOT/gpurun_out/r4f/ov_$mode.log 2>&1 || exit 1
  (cd $GRAFT_REPO_ROOT && grep "mode" gpurun_out/r4f/ov_$mode.log | tail -1 && python3 tools/prof_summary.py gpurun_out/r4f/ov_$mode --by-grid > gpurun_out/r4f/ov_${mode}_kernels.txt && head -14 gpurun_out/r4f/ov_${mode}_kernels.txt)
  find $GRAFT_REPO_ROOT/gpurun_out/r4f/ov_$mode -name "*.db" -delete
done
