#!/bin/bash
# round 6 job b: the tests touched by the round-6 fixes (grid-cap / split-K knob split,
# chunked large shards, bf16 bounds in ulps, FusedSGD coef), then the strong-scaling legs.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6_b
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread -m gpu \
  tests/test_scan_gpu.py tests/test_attention_gpu.py tests/test_gemm_gpu.py \
  "tests/test_model_gpu.py::test_bert_long_512_matches_reference" tests/test_train_gpu.py \
  > $O/pytest.log 2>&1
rc=$?
grep -E "ulps|passed|failed|FAILED|Error" $O/pytest.log | tail -60
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --part strong --no-cpu-baseline > $O/bench_strong.log 2>&1 || { tail $O/bench_strong.log; exit 1; }
tail -1 $O/bench_strong.log | cut -c1-3000
cp gpurun_out/bench_detail.json $O/bench_strong_detail.json 2>/dev/null
true
