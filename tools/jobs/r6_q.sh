#!/bin/bash
# round 6 job q: a rehearsal of the driver's N-rank bench on the 1-GPU box: bench.py --gpus 2
# with IRC_DIST_BACKEND=gloo (both ranks on the one GPU), every part, short runs -- the
# launcher, the DP training steps (LSTM and --model BERT), the sharded and strong-scaling
# retrieval legs and the max-over-ranks JSON line, end to end.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6_q
mkdir -p $O
export PYTHONUNBUFFERED=1 IRC_DIST_BACKEND=gloo
for part in train bert scan strong; do
  timeout -k 10 400 python bench.py --gpus 2 --part $part --steps 3 --warmup 1 --no-cpu-baseline \
    > $O/ws2_$part.log 2>&1 || { tail -20 $O/ws2_$part.log; exit 1; }
  tail -1 $O/ws2_$part.log | cut -c1-300
done
