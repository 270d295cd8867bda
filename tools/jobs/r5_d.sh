#!/bin/bash
# round 5 job d: bench line with the step-level roofline; main.py end to end with the
# batched pair sampler, against the synthetic train leg on the same box
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u bench.py > gpurun_out/r5_d_bench.log 2>&1 || exit $?
tail -1 gpurun_out/r5_d_bench.log
timeout -k 10 400 python -u tools/e2e_train.py --steps 80 > gpurun_out/r5_d_e2e.log 2>&1 || exit $?
grep -E "end-to-end|host time|host tokenizer" gpurun_out/r5_d_e2e.log
timeout -k 10 300 python -u bench.py --part train --no-cpu-baseline > gpurun_out/r5_d_bench_train.log 2>&1 || exit $?
tail -1 gpurun_out/r5_d_bench_train.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('train leg', d['value'], d['ms_per_step'])"
