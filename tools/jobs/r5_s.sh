#!/bin/bash
# round 5 job s: BERT-alone / heads-alone / overlapped step (host_time) and the cluster
# recurrences' run-to-run reproducibility on the current code
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/host_time.py --steps 30 > gpurun_out/r5_s_host_time.log 2>&1 || exit $?
grep -E "alone|wall" gpurun_out/r5_s_host_time.log
timeout -k 10 300 python -u tools/lstm_coop_repro.py --n 4 > gpurun_out/r5_s_repro.log 2>&1 || exit $?
tail -6 gpurun_out/r5_s_repro.log
bash tools/jobs/r5_t.sh
