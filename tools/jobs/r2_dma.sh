# DMA ownership A/B: release (group 0 stages both B halves, each group waits two sections
# after issuing) vs the splitb variant (B split by group, group 1 waits in the issuing section).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py tests/test_scan_gpu.py tests/test_scan_fp8_gpu.py tests/test_fp8_encoder_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_dma.log 2>&1 || { tail -30 gpurun_out/pytest_dma.log; exit 1; }
tail -1 gpurun_out/pytest_dma.log
V=information-retrieval-with-contrastive-learning_amd/irc_amd/lib/variants/splitb.so
for rep in 1 2; do
  IRC_LIB_PATH=$V timeout -k 10 200 python tools/gemm_bench.py --iters 50 > gpurun_out/gemm_old$rep.txt 2>&1 || exit 1
  timeout -k 10 200 python tools/gemm_bench.py --iters 50 > gpurun_out/gemm_new$rep.txt 2>&1 || exit 1
done
paste gpurun_out/gemm_old1.txt gpurun_out/gemm_new1.txt gpurun_out/gemm_old2.txt gpurun_out/gemm_new2.txt | awk -F'\t' '{printf "%-40s", substr($1,1,40); for(i=1;i<=NF;i++){n=split($i,a," "); for(j=1;j<=n;j++) if(a[j]=="us") printf " %8s", a[j-1]}; print ""}'
for rep in 1 2; do
  IRC_LIB_PATH=$V timeout -k 10 300 python bench.py --part train --no-cpu-baseline > gpurun_out/train_old$rep.log 2>&1 || exit 1
  timeout -k 10 300 python bench.py --part train --no-cpu-baseline > gpurun_out/train_new$rep.log 2>&1 || exit 1
done
for f in old1 new1 old2 new2; do echo $f $(grep -o '"value": [0-9.]*' gpurun_out/train_$f.log | head -1); done
exit 0
