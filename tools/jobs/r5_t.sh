#!/bin/bash
# round 5 job t: the heads' weight-gradient GEMMs alone, time and HBM traffic per launch
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 200 python -u tools/dw_bench.py > gpurun_out/r5_t_dw.log 2>&1 || exit $?
grep "us" gpurun_out/r5_t_dw.log
export TMPDIR=/tmp
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r5_t_prof -o run -- python3 $R/tools/dw_bench.py --iters 5 > $R/gpurun_out/r5_t_prof.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/r5_t_fetch -o run -- python3 $R/tools/dw_bench.py --iters 5 > $R/gpurun_out/r5_t_fetch.log 2>&1 || exit $?
cd $R
python3 tools/trace_top.py gpurun_out/r5_t_prof --top 12
