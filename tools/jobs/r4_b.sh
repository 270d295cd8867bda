# Round 4 job b: scan + GEMM GPU tests (single-pass GEMM filter, chunk key, GELU),
# single-pass vs sampled A/B, gemm_big chunk key A/B + LDS counters, hipBLASLt calibration.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r4b
V=$GRAFT_REPO_ROOT/information-retrieval-with-contrastive-learning_amd/irc_amd/lib/variants/oldswz.so
timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py tests/test_scan_gpu.py tests/test_scan_fp8_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r4b/tests.log 2>&1 || { tail -40 gpurun_out/r4b/tests.log; exit 1; }
tail -2 gpurun_out/r4b/tests.log
timeout -k 10 300 python tools/scan_ppl_ab.py > gpurun_out/r4b/ppl_ab.txt 2>&1 || { tail -20 gpurun_out/r4b/ppl_ab.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r4b/ppl_ab.txt
for fp8 in "" "--fp8"; do
  for smp in 1 0; do
    D=1024; [ -n "$fp8" ] && D=768
    IRC_SCAN_PP_SAMPLE=$smp timeout -k 10 200 python tools/scan_call_prof.py --n 625000 --d $D --q 2048 $fp8 > gpurun_out/r4b/c45_$smp$fp8.txt 2>&1 || exit 1
    echo "pp_sample=$smp $(grep -v amdgpu.ids gpurun_out/r4b/c45_$smp$fp8.txt)"
  done
done
SH=qkv,attn_out+res,ffn1+gelu,ffn1+bias,ffn2+res,lstm_xp_l0,square4k
timeout -k 10 200 python tools/gemm_bench.py --only $SH --duo ab > gpurun_out/r4b/gemm_new.txt 2>&1 || exit 1
IRC_LIB_PATH=$V timeout -k 10 200 python tools/gemm_bench.py --only $SH > gpurun_out/r4b/gemm_old.txt 2>&1 || exit 1
for f in gemm_new gemm_old; do echo "== $f"; grep -v amdgpu.ids gpurun_out/r4b/$f.txt; done
timeout -k 10 200 python tools/torch_gemm_ref.py > gpurun_out/r4b/torch_ref.txt 2>&1; grep -v amdgpu.ids gpurun_out/r4b/torch_ref.txt
cd /tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r4b/pmc_new/p1 -o run -- \
  python3 $GRAFT_REPO_ROOT/tools/gemm_bench.py --iters 3 --only qkv,attn_out+res,ffn2+res > $GRAFT_REPO_ROOT/gpurun_out/r4b/pmc.log 2>&1 || exit 1
cd "$GRAFT_REPO_ROOT" && echo "== NEW" && python3 tools/pmc_table.py gpurun_out/r4b/pmc_new gemm_big
