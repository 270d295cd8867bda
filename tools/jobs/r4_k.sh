# Round 4 job k: FFN1 on the big-tile 16x16x32 kernel vs the ping-pong one; the C4 / C5
# retrieval call against the threshold-sample size, and the C4 call's kernel breakdown.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/r4k
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_qkv_attn_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 120 python tools/qkv_attn_bench.py > $OUT/qkv_attn.txt 2>&1 || exit 1
grep -v amdgpu $OUT/qkv_attn.txt
for r in 1 2; do
  timeout -k 10 200 python tools/gemm_bench.py --only ffn1+gelu,ffn1+bias,ffn2+res > $OUT/ffn_pp_$r.txt 2>&1 || exit 1
  IRC_GEMM_PP=0 timeout -k 10 200 python tools/gemm_bench.py --only ffn1+gelu,ffn1+bias,ffn2+res > $OUT/ffn_big_$r.txt 2>&1 || exit 1
done
for f in ffn_pp_1 ffn_big_1 ffn_pp_2 ffn_big_2; do echo "== $f"; grep -v amdgpu $OUT/$f.txt; done
for dv in 8 16 32; do
  IRC_SCAN_SAMPLE_DIV=$dv timeout -k 10 200 python tools/scan_call_prof.py --n 625000 --d 1024 --q 2048 --reps 10 > $OUT/c4_div$dv.txt 2>&1 || exit 1
  IRC_SCAN_SAMPLE_DIV=$dv timeout -k 10 200 python tools/scan_call_prof.py --n 625000 --d 768 --q 2048 --fp8 --reps 10 > $OUT/c5_div$dv.txt 2>&1 || exit 1
  echo "div=$dv"; grep -h "us per call" $OUT/c4_div$dv.txt $OUT/c5_div$dv.txt
done
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/c4_trace -o run -- \
  python3 $GRAFT_REPO_ROOT/tools/scan_call_prof.py --n 625000 --d 1024 --q 2048 --reps 10 > $OUT/c4_trace.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && python3 tools/prof_summary.py $OUT/c4_trace > $OUT/c4_trace_kernels.txt && head -12 $OUT/c4_trace_kernels.txt
find $OUT -name "*.db" -delete
cd /tmp
for s in qkv ffn1+gelu ffn2+res square4k; do
  t=$(echo $s | tr '+^' 'p_')
  timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE --output-format csv -d $OUT/clk_$t -o run -- \
    python3 $GRAFT_REPO_ROOT/tools/gemm_bench.py --only $s --iters 20 > $OUT/clk_$t.log 2>&1 || { echo "clock pass $s failed"; exit 1; }
  (cd $GRAFT_REPO_ROOT && python3 tools/pmc_clock.py $OUT/clk_$t $OUT/clk_$t.log)
done
find $OUT -name "*.csv" -size +2M -delete
