# LDS counters of the big-tile / ping-pong GEMMs on the BERT shapes (one --pmc pass each).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/lds
mkdir -p $OUT
cd /tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY --output-format csv -d $OUT/p1 -o run -- \
  python3 $GRAFT_REPO_ROOT/tools/gemm_bench.py --iters 3 --only qkv,attn_out+res,ffn1+gelu,ffn2+res > $OUT/p1.log 2>&1 || { tail -20 $OUT/p1.log; exit 1; }
cd "$GRAFT_REPO_ROOT" && python3 tools/pmc_table.py $OUT gemm 2>&1 | tail -60
