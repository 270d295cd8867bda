#!/bin/bash
# Round 6 closing run on the final code: the whole GPU suite, smoke, bench.py (default line:
# every leg, CPU baselines included), rocprofv3 kernel-trace summaries of the train, scan_c2,
# scan_c3 and bert parts, and main.py end to end.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${R6FIN:-r6fin}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/ \
  > $O/pytest_gpu.log 2>&1
rc=$?
tail -2 $O/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/pytest_gpu.log | head; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 900 python bench.py > $O/bench.log 2>&1 || { tail $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-600
cp gpurun_out/bench_detail.json $O/bench_detail.json 2>/dev/null
export TMPDIR=/tmp
cd /tmp || exit 1
for part in train scan_c2 scan_c3 bert; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_$part -o run -- \
    python3 $R/bench.py --part $part --steps 10 --warmup 3 --no-cpu-baseline > $O/prof_$part.log 2>&1 \
    || { tail $O/prof_$part.log; exit 1; }
done
cd $R || exit 1
for part in train scan_c2 scan_c3 bert; do
  python3 tools/prof_summary.py $O/prof_$part --top=40 > $O/${part}_kernels.txt && head -6 $O/${part}_kernels.txt
done
timeout -k 10 400 python -u tools/e2e_train.py --steps 80 > $O/e2e.log 2>&1 || { tail $O/e2e.log; exit 1; }
grep -E "end-to-end" $O/e2e.log
