#!/bin/bash
# round 6 job t: where a batch padded to L = 65 loses against L = 64 (9.7 vs 8.4 ms a C2
# step): kernel traces of tools/e2e_probe.py --by-len at each length, summarised.
# (Run on the code with the since-reverted tail grid cap, profiles/r06_s/.)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6_t
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for L in 64 65; do
  cd /tmp || exit 1
  timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $O/prof_$L -o run -- \
    python3 $R/tools/e2e_probe.py --by-len --lens $L --steps 40 > $O/probe_$L.log 2>&1 \
    || { tail $O/probe_$L.log; exit 1; }
  cd $R || exit 1
  python3 tools/prof_summary.py $O/prof_$L --top=60 > $O/kernels_$L.txt
  grep "L=" $O/probe_$L.log
done
rm -rf $O/prof_64 $O/prof_65
