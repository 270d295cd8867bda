# Round 4 job v: fused QKV + attention epilogue with packed staging stores and transposed
# V reads: exactness tests and the layer timing.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/r4v
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_qkv_attn_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for r in 1 2 3; do timeout -k 10 100 python tools/qkv_attn_bench.py --iters 30 >> $OUT/qa.txt 2>&1 || exit 1; done
grep -v amdgpu $OUT/qa.txt
