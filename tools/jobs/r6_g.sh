#!/bin/bash
# round 6 job g: HBM traffic (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes) of every bench
# part's dominant kernel family on the round-6 code: the C2 scan filter and the GEMMs of the
# C2, C4 (BERT-large), --model BERT and C5 (MX-fp8) training legs.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
PMC_PARTS="scan_c2 train train_c4 bert train_fp8" timeout -k 10 1500 bash tools/pmc_traffic.sh > gpurun_out/pmc_r6.log 2>&1
rc=$?
tail -12 gpurun_out/pmc_r6.log
ls gpurun_out/pmc/*.json
exit $rc
