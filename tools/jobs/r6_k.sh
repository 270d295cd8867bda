#!/bin/bash
# round 6 job k: fused QKV + attention against the two-launch form at the encoder's real
# batch (B = 512 sequences, a C2 / C4 micro-batch; B = 504 the split chunk at L = 65) over
# the L grid a batch's joint padding lands on, for the release selection (slots; packed at
# L in [29, 32]) and for the A/B build with packed tiles wherever they hold more sequences.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6_k
mkdir -p $O
export PYTHONUNBUFFERED=1
V=$R/information-retrieval-with-contrastive-learning_amd/irc_amd/lib/variants
LENS=16,20,24,28,30,32,34,36,40,44,48,52,56,60,62,63,64,65,68,72,76,80,85,88,92,96,100,104,112,120,128
for v in release pack_any; do
  if [ $v = release ]; then unset IRC_LIB_PATH; else export IRC_LIB_PATH=$V/qkv_pack_any.so; fi
  timeout -k 10 400 python -u tools/qkv_attn_bench.py --iters 20 --b 512 --lens $LENS \
    > $O/$v.log 2>&1 || { tail $O/$v.log; exit 1; }
  timeout -k 10 100 python -u tools/qkv_attn_bench.py --iters 20 --b 504 --lens 65 \
    >> $O/$v.log 2>&1 || { tail $O/$v.log; exit 1; }
  echo "== $v"; grep "H=" $O/$v.log | awk '{print $2, $3, $4, $5}' | paste - - - -
done
