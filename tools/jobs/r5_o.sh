#!/bin/bash
# round 5 job o: where a cluster-forward step's 4.5 us go (phase stamps, diagnostic build)
set -o pipefail
mkdir -p gpurun_out
V=$GRAFT_REPO_ROOT/information-retrieval-with-contrastive-learning_amd/irc_amd/lib/variants/coopstamps.so
IRC_LIB_PATH=$V timeout -k 10 200 python -u tools/coop_stamps.py --bg 32 > gpurun_out/r5_o_stamps32.log 2>&1 || { tail gpurun_out/r5_o_stamps32.log; exit 1; }
IRC_LIB_PATH=$V timeout -k 10 200 python -u tools/coop_stamps.py --bg 64 > gpurun_out/r5_o_stamps64.log 2>&1 || { tail gpurun_out/r5_o_stamps64.log; exit 1; }
grep -v Warn gpurun_out/r5_o_stamps32.log gpurun_out/r5_o_stamps64.log
