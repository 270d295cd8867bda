#!/bin/bash
# round 5 job r: the heads step alone -- wall and its kernels (rocprofv3 kernel trace)
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 200 python -u tools/heads_alone.py > gpurun_out/r5_r_heads.log 2>&1 || exit $?
grep heads gpurun_out/r5_r_heads.log
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r5_r_prof -o run -- python3 $R/tools/heads_alone.py --steps 20 > $R/gpurun_out/r5_r_prof.log 2>&1 || exit $?
cd $R
python3 tools/trace_top.py gpurun_out/r5_r_prof --top 40
