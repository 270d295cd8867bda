# Round 4 job i: QKV projection + attention in one launch (irc_qkv_attention): parity tests,
# the fused vs two-launch layer interleaved, and the C2 / C4 steps with and without it.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r4i
timeout -k 10 400 python -u -m pytest tests/test_qkv_attn_gpu.py tests/test_ln_fold_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r4i/tests.log 2>&1 || { tail -40 gpurun_out/r4i/tests.log; exit 1; }
tail -1 gpurun_out/r4i/tests.log
timeout -k 10 120 python tools/qkv_attn_bench.py > gpurun_out/r4i/qkv_attn.txt 2>&1 || exit 1
timeout -k 10 120 python tools/qkv_attn_bench.py --h 1024 >> gpurun_out/r4i/qkv_attn.txt 2>&1 || exit 1
grep -v amdgpu gpurun_out/r4i/qkv_attn.txt
for r in 1 2; do
  for f in 0 1; do
    IRC_QKV_ATTN=$f timeout -k 10 200 python bench.py --part train --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/r4i/train_${f}_$r.log 2>&1 || exit 1
    python3 - gpurun_out/r4i/train_${f}_$r.log $f <<'PY'
import json, sys
d = json.loads([x for x in open(sys.argv[1]) if x.startswith('{')][-1])
print("train qkv_attn=%s" % sys.argv[2], round(d["value"]), round(d["ms_per_step"], 3), round(d["roofline"]["frac"], 4))
PY
  done
done
for f in 0 1; do
  IRC_QKV_ATTN=$f timeout -k 10 300 python bench.py --part train_c4 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r4i/c4_${f}.log 2>&1 || exit 1
  python3 - gpurun_out/r4i/c4_${f}.log $f <<'PY'
import json, sys
d = json.loads([x for x in open(sys.argv[1]) if x.startswith('{')][-1])
print("c4 qkv_attn=%s" % sys.argv[2], round(d["value"]), round(d["ms_per_step"], 3))
PY
done
cd /tmp
IRC_QKV_ATTN=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r4i/bert_fused -o run -- \
  python3 $GRAFT_REPO_ROOT/tools/overlap_prof.py --mode bert --steps 20 > $GRAFT_REPO_ROOT/gpurun_out/r4i/bert_fused.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && grep "mode" gpurun_out/r4i/bert_fused.log | tail -1 && python3 tools/prof_summary.py gpurun_out/r4i/bert_fused --by-grid > gpurun_out/r4i/bert_fused_kernels.txt && head -10 gpurun_out/r4i/bert_fused_kernels.txt
find gpurun_out/r4i/bert_fused -name "*.db" -delete
