# HBM traffic of the train part's bf16 GEMMs with the grouped tile order (IRC_GEMM_GROUP_M=8):
# does the order cut the weight-tile re-fetch? (compare profiles/pmc_gemm_bf16.json)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmcg
mkdir -p $OUT
export IRC_GEMM_GROUP_M=8
cd /tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $c --output-format csv -d $OUT/train_$c -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --part train --steps 3 --warmup 1 --no-cpu-baseline \
    > $OUT/train_$c.log 2>&1 || { echo "pass $c failed"; exit 1; }
done
cd "$GRAFT_REPO_ROOT" || exit 1
GEMM='gemm_big_kernel<|gemm_kernel<unsigned short|gemm_pp_kernel<(true|false), (true|false), [a-z ]+, [0-6], false>'
python3 tools/pmc_summary.py $OUT/train_FETCH_SIZE $OUT/train_WRITE_SIZE "$GEMM" gemm_bf16_group8 --out $OUT \
  --note "all bf16 GEMM dispatches of bench.py --part train with IRC_GEMM_GROUP_M=8" || exit 1
exit 0
