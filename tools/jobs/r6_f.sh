#!/bin/bash
# round 6 job f: checkpoint -- the whole GPU suite on the round-6 code (interleaved scan DMA by
# default, knobs removed, overlapped BERT weight gradients, batched transposed casts), the
# --model BERT leg, and the scan Q sweep on the C2 / C3 shards.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6_f
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/ \
  > $O/pytest_gpu.log 2>&1
rc=$?
tail -2 $O/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/pytest_gpu.log | head; exit $rc; }
timeout -k 10 300 python bench.py --part bert --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_bert.log 2>&1 || { tail $O/bench_bert.log; exit 1; }
tail -1 $O/bench_bert.log | cut -c1-400
for n in 250000 100000; do
  timeout -k 10 120 python tools/scan_bench.py --n $n --reps 30 > $O/scan_n$n.log 2>&1 || { tail $O/scan_n$n.log; exit 1; }
  grep filter $O/scan_n$n.log
done
