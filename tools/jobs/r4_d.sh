# Round 4 job d: breakdown of the single-pass scan call (kernel trace), the gemm_big chunk
# key A/B + LDS counters, and the hipBLASLt calibration of the BERT shapes.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r4d
V=$GRAFT_REPO_ROOT/information-retrieval-with-contrastive-learning_amd/irc_amd/lib/variants/oldswz.so
cd /tmp
for m in 65 999; do
  IRC_SCAN_PPL_MINQ=$m timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r4d/scan_$m -o run -- \
    python3 $GRAFT_REPO_ROOT/tools/scan_call_prof.py --n 100000 --d 768 --q 256 --reps 50 > $GRAFT_REPO_ROOT/gpurun_out/r4d/scan_$m.log 2>&1 || exit 1
  (cd $GRAFT_REPO_ROOT && grep -v amdgpu gpurun_out/r4d/scan_$m.log | tail -1 && python3 tools/prof_summary.py gpurun_out/r4d/scan_$m > gpurun_out/r4d/scan_${m}_kernels.txt && head -8 gpurun_out/r4d/scan_${m}_kernels.txt)
  find $GRAFT_REPO_ROOT/gpurun_out/r4d/scan_$m -name "*.db" -delete
done
cd "$GRAFT_REPO_ROOT"
SH=qkv,attn_out+res,ffn1+gelu,ffn1+bias,ffn2+res,lstm_xp_l0,square4k
for r in 1 2; do
  timeout -k 10 200 python tools/gemm_bench.py --only $SH > gpurun_out/r4d/gemm_new_$r.txt 2>&1 || exit 1
  IRC_LIB_PATH=$V timeout -k 10 200 python tools/gemm_bench.py --only $SH > gpurun_out/r4d/gemm_old_$r.txt 2>&1 || exit 1
done
for f in gemm_new_1 gemm_old_1 gemm_new_2 gemm_old_2; do echo "== $f"; grep -v amdgpu gpurun_out/r4d/$f.txt; done
timeout -k 10 300 python tools/torch_gemm_ref.py > gpurun_out/r4d/torch_ref.txt 2>&1; grep -v amdgpu gpurun_out/r4d/torch_ref.txt
cd /tmp
for m in new old; do
  if [ $m = old ]; then export IRC_LIB_PATH=$V; else unset IRC_LIB_PATH; fi
  timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r4d/pmc_$m/p1 -o run -- \
    python3 $GRAFT_REPO_ROOT/tools/gemm_bench.py --iters 3 --only qkv,attn_out+res,ffn2+res > $GRAFT_REPO_ROOT/gpurun_out/r4d/pmc_$m.log 2>&1 || exit 1
done
unset IRC_LIB_PATH
cd "$GRAFT_REPO_ROOT" && for m in new old; do echo "== LDS $m"; python3 tools/pmc_table.py gpurun_out/r4d/pmc_$m gemm_big; done
