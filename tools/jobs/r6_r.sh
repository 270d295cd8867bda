#!/bin/bash
# round 6 job r: where main.py end to end loses against the train leg -- rocprofv3 kernel
# traces of both (80 e2e steps; the train part's 10 + 3), summarised per kernel.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6_r
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
cd /tmp || exit 1
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $O/prof_e2e -o run -- \
  python3 $R/tools/e2e_train.py --steps 80 > $O/e2e.log 2>&1 || { tail $O/e2e.log; exit 1; }
cd $R || exit 1
python3 tools/prof_summary.py $O/prof_e2e --top=45 > $O/e2e_kernels.txt && head -30 $O/e2e_kernels.txt
grep -E "end-to-end|histogram" $O/e2e.log
