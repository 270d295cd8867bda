# Grouped tile order A/B (IRC_GEMM_GROUP_M) on the GEMM microbench and the C2 train step.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
IRC_GEMM_GROUP_M=8 timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_gemm.log 2>&1 || { tail -30 gpurun_out/pytest_gemm.log; exit 1; }
tail -1 gpurun_out/pytest_gemm.log
for gm in 0 4 8 16 0 8; do
  IRC_GEMM_GROUP_M=$gm timeout -k 10 200 python tools/gemm_bench.py --iters 50 > gpurun_out/gemm_g$gm.txt 2>&1 || exit 1
  cp gpurun_out/gemm_g$gm.txt gpurun_out/gemm_g${gm}_$(date +%s).txt
done
paste gpurun_out/gemm_g0.txt gpurun_out/gemm_g4.txt gpurun_out/gemm_g8.txt gpurun_out/gemm_g16.txt | awk -F'\t' '{printf "%-40s", substr($1,1,40); for(i=1;i<=NF;i++){n=split($i,a," "); for(j=1;j<=n;j++) if(a[j]=="us") printf " %8s", a[j-1]}; print ""}'
for gm in 0 8 0 8; do
  IRC_GEMM_GROUP_M=$gm timeout -k 10 300 python bench.py --part train --no-cpu-baseline > gpurun_out/train_g$gm.log 2>&1 || exit 1
  echo g$gm $(grep -o '"value": [0-9.]*' gpurun_out/train_g$gm.log | head -1)
done
exit 0
