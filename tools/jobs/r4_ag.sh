# Round 4 job ag: the cluster path skips the single-CU W_hh packs -- LSTM / model / train
# GPU tests, heads-alone step, the train leg.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/r4ag
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_lstm_mfma_gpu.py tests/test_model_gpu.py tests/test_train_gpu.py tests/test_configs_gpu.py > $OUT/tests.log 2>&1 \
  || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 300 python tools/host_time.py --steps 30 > $OUT/host_time.log 2>&1 || { tail -20 $OUT/host_time.log; exit 1; }
grep -v amdgpu $OUT/host_time.log | tail -3
timeout -k 10 400 python bench.py --part train > $OUT/bench_train.log 2>&1 || { tail -20 $OUT/bench_train.log; exit 1; }
grep '^{' $OUT/bench_train.log | tail -1 | cut -c1-300
