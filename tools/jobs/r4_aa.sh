# Round 4 job aa: hprev written by the cluster forward (no separate shift pass) --
# the LSTM / heads / training GPU tests, then the train leg and the heads-alone step on
# one box, then main.py end to end with the DataLoader wait timed.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/r4aa
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_lstm_mfma_gpu.py tests/test_model_gpu.py tests/test_train_gpu.py > $OUT/tests.log 2>&1 \
  || { tail -30 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
timeout -k 10 300 python tools/host_time.py --steps 30 > $OUT/host_time.log 2>&1 || { tail -20 $OUT/host_time.log; exit 1; }
cat $OUT/host_time.log | grep -v amdgpu
timeout -k 10 400 python bench.py --part train > $OUT/bench_train.log 2>&1 || { tail -20 $OUT/bench_train.log; exit 1; }
grep '^{' $OUT/bench_train.log | tail -1 | cut -c1-400
timeout -k 10 600 python tools/e2e_train.py --steps 80 > $OUT/e2e.log 2>&1 || { tail -20 $OUT/e2e.log; exit 1; }
grep -v amdgpu $OUT/e2e.log | grep -v "it/s\|Warning\|return _m\|ret = " | tail -8
