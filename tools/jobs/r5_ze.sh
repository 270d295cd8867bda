#!/bin/bash
# round 5 job ze: GPU tests of the touched paths; C2 train leg with the head's dX GEMM capped
# too (release) vs every split GEMM capped (variants/split128.so), interleaved; retrieval legs
# at three batches in flight without graphs
set -o pipefail
mkdir -p gpurun_out
V=$GRAFT_REPO_ROOT/information-retrieval-with-contrastive-learning_amd/irc_amd/lib/variants/split128.so
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_scan_gpu.py tests/test_gemm_gpu.py tests/test_lstm_mfma_gpu.py tests/test_train_gpu.py \
  > gpurun_out/r5_ze_tests.log 2>&1 || { tail -30 gpurun_out/r5_ze_tests.log; exit 1; }
tail -1 gpurun_out/r5_ze_tests.log
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --part train --no-cpu-baseline > gpurun_out/r5_ze_rel_$i.log 2>&1 || exit $?
  echo "rel     $(tail -1 gpurun_out/r5_ze_rel_$i.log | cut -c95-175)"
  IRC_LIB_PATH=$V timeout -k 10 300 python bench.py --part train --no-cpu-baseline > gpurun_out/r5_ze_all_$i.log 2>&1 || exit $?
  echo "all128  $(tail -1 gpurun_out/r5_ze_all_$i.log | cut -c95-175)"
done
timeout -k 10 500 python bench.py --part scan --no-cpu-baseline > gpurun_out/r5_ze_scan.log 2>&1 || { tail gpurun_out/r5_ze_scan.log; exit 1; }
cp gpurun_out/bench_detail.json gpurun_out/r5_ze_scan_detail.json
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/r5_ze_scan_detail.json"))
for k, v in d.items():
    if k.startswith("retrieval") and isinstance(v, dict):
        print(k, round(v["value"]), v["unit"], round(v["ms_per_batch"] * 1e3, 1), "us/batch")
PY
