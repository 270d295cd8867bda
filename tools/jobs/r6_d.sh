#!/bin/bash
# round 6 job d: the --model BERT leg itemised -- a kernel trace of the bench part (fwd,
# bwd, optimizer) with every kernel family's time per step.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6_d
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_bert_train_gpu.py tests/test_dist_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 400 python tools/bert_wgrad_ab.py --steps 10 --reps 3 --cap 0 128 > $O/wgrad_ab.log 2>&1 || { tail $O/wgrad_ab.log; exit 1; }
cat $O/wgrad_ab.log
timeout -k 10 300 python bench.py --part bert --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_bert.log 2>&1 || { tail $O/bench_bert.log; exit 1; }
tail -1 $O/bench_bert.log | cut -c1-600
export TMPDIR=/tmp
cd /tmp || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_bert -o run -- \
  python3 $R/bench.py --part bert --steps 10 --warmup 3 --no-cpu-baseline > $O/prof_bert.log 2>&1 \
  || { tail $O/prof_bert.log; exit 1; }
cd $R || exit 1
python3 tools/prof_summary.py $O/prof_bert --top=70 > $O/bert_kernels.txt && head -72 $O/bert_kernels.txt
# the frozen encoder alone, bf16 against MX-fp8 weights (C5), per-kernel split
timeout -k 10 300 python tools/encode_bench.py --iters 20 > $O/encode_bench.log 2>&1 || { tail $O/encode_bench.log; exit 1; }
cat $O/encode_bench.log
