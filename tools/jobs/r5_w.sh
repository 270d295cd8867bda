#!/bin/bash
# round 5 job w: FFN1 + GELU (and the other BERT shapes) on the 256x256 ping-pong kernel
# against the 256x384 big-tile kernel (IRC_GEMM_PP=0), interleaved
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 200 python -u tools/gemm_bench.py --only qkv,attn_out+res,ffn1+gelu,ffn2+res --iters 30 > gpurun_out/r5_w_pp_$i.log 2>&1 || exit $?
  sed 's/^/pp  /' gpurun_out/r5_w_pp_$i.log | grep epi
  IRC_GEMM_PP=0 timeout -k 10 200 python -u tools/gemm_bench.py --only qkv,attn_out+res,ffn1+gelu,ffn2+res --iters 30 > gpurun_out/r5_w_big_$i.log 2>&1 || exit $?
  sed 's/^/big /' gpurun_out/r5_w_big_$i.log | grep epi
done
