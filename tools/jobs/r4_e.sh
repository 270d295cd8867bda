# Round 4 job e: residual-epilogue prefetch A/B of the big-tile kernel (base / RPRE / RPRE2).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r4e
L=$GRAFT_REPO_ROOT/information-retrieval-with-contrastive-learning_amd/irc_amd/lib
SH=attn_out+res,ffn2+res,qkv
for r in 1 2; do
  for v in base rpre rpre2; do
    if [ $v = base ]; then unset IRC_LIB_PATH; else export IRC_LIB_PATH=$L/variants/$v.so; fi
    timeout -k 10 120 python tools/gemm_bench.py --only $SH > gpurun_out/r4e/gemm_${v}_$r.txt 2>&1 || exit 1
    echo "== $v $r"; grep -v amdgpu gpurun_out/r4e/gemm_${v}_$r.txt
  done
done
timeout -k 10 300 python tools/host_time.py --steps 30 > gpurun_out/r4e/host_time.txt 2>&1 || exit 1
grep -v amdgpu gpurun_out/r4e/host_time.txt
timeout -k 10 200 python tools/scan_call_prof.py --n 625000 --d 1024 --q 2048 > gpurun_out/r4e/c4.txt 2>&1 && grep -v amdgpu gpurun_out/r4e/c4.txt
