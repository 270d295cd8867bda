# Round 4: A/B of the gemm_big chunk key (new (r >> 1) & 7 vs variants/oldswz.so).
# gemm_big chunk key (r >> 1) & 7 vs the round-2 r & 7: GEMM / encoder / config tests, LDS
# counters, BERT-shape A/B and the C2 / C4 step A/B on one box.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/swz
V=$GRAFT_REPO_ROOT/information-retrieval-with-contrastive-learning_amd/irc_amd/lib/variants/oldswz.so
timeout -k 10 500 python -u -m pytest tests/test_gemm_gpu.py tests/test_encoder_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/swz/tests.log 2>&1 || { tail -30 gpurun_out/swz/tests.log; exit 1; }
tail -1 gpurun_out/swz/tests.log
SH=qkv,attn_out+res,ffn2+res,lstm_xp_l0,lstm_xp_l12
for r in 1; do
  timeout -k 10 200 python tools/gemm_bench.py --only $SH > gpurun_out/swz/new_$r.txt 2>&1 || exit 1
  IRC_LIB_PATH=$V timeout -k 10 200 python tools/gemm_bench.py --only $SH > gpurun_out/swz/old_$r.txt 2>&1 || exit 1
done
for f in new_1 old_1; do echo "== $f"; grep -v amdgpu.ids gpurun_out/swz/$f.txt; done
for r in 1; do
  for m in new old; do
    if [ $m = old ]; then export IRC_LIB_PATH=$V; else unset IRC_LIB_PATH; fi
    timeout -k 10 200 python bench.py --part train --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/swz/train_${m}_$r.log 2>&1 || exit 1
    python - gpurun_out/swz/train_${m}_$r.log $m <<'PY'
import json, sys
d = json.loads([x for x in open(sys.argv[1]) if x.startswith('{')][0])
print("train", sys.argv[2], round(d["value"]), round(d["ms_per_step"], 3), round(d["roofline"]["frac"], 4))
PY
  done
done
unset IRC_LIB_PATH
cd /tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/swz/pmc/p1 -o run -- \
  python3 $GRAFT_REPO_ROOT/tools/gemm_bench.py --iters 3 --only qkv,attn_out+res,ffn2+res > $GRAFT_REPO_ROOT/gpurun_out/swz/pmc.log 2>&1 || exit 1
cd "$GRAFT_REPO_ROOT" && python3 tools/pmc_table.py gpurun_out/swz/pmc gemm_big
cd /tmp
IRC_LIB_PATH=$V timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/swz/pmc_old/p1 -o run -- \
  python3 $GRAFT_REPO_ROOT/tools/gemm_bench.py --iters 3 --only qkv,attn_out+res,ffn2+res > $GRAFT_REPO_ROOT/gpurun_out/swz/pmc_old.log 2>&1 || exit 1
cd "$GRAFT_REPO_ROOT" && echo "== OLD" && python3 tools/pmc_table.py gpurun_out/swz/pmc_old gemm_big
cd "$GRAFT_REPO_ROOT" && timeout -k 10 200 python tools/torch_gemm_ref.py > gpurun_out/swz/torch_ref.txt 2>&1; grep -v amdgpu.ids gpurun_out/swz/torch_ref.txt
