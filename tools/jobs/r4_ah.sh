# Round 4 job ah: cluster height 48 (RB = 3) against 32 -- bit identity and latency of the
# recurrences, the LSTM / train GPU tests at 48, and the overlapped train leg interleaved.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/r4ah
mkdir -p $OUT
timeout -k 10 300 python tools/lstm_coop_bench.py --ab IRC_LSTM_COOP_RB=2,IRC_LSTM_COOP_RB=3 > $OUT/lstm_rb_ab.log 2>&1 || { tail -20 $OUT/lstm_rb_ab.log; exit 1; }
grep round $OUT/lstm_rb_ab.log
timeout -k 10 300 python tools/lstm_coop_bench.py --b 40 --l 7 --iters 5 --ab IRC_LSTM_COOP_RB=2,IRC_LSTM_COOP_RB=3 > $OUT/lstm_rb_ab_small.log 2>&1 || { tail -20 $OUT/lstm_rb_ab_small.log; exit 1; }
grep round $OUT/lstm_rb_ab_small.log
IRC_LSTM_COOP_RB=3 timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_lstm_mfma_gpu.py tests/test_model_gpu.py tests/test_train_gpu.py > $OUT/tests_rb3.log 2>&1 \
  || { tail -30 $OUT/tests_rb3.log; exit 1; }
tail -1 $OUT/tests_rb3.log
for r in 2 3 2 3; do
IRC_LSTM_COOP_RB=$r timeout -k 10 400 python bench.py --part train > $OUT/bench_train_rb$r.log 2>&1 || { tail -20 $OUT/bench_train_rb$r.log; exit 1; }
echo "rb=$r $(grep '^{' $OUT/bench_train_rb$r.log | tail -1 | cut -c90-150)"
done
IRC_LSTM_COOP_RB=3 timeout -k 10 300 python tools/host_time.py --steps 30 > $OUT/host_time_rb3.log 2>&1 || { tail -20 $OUT/host_time_rb3.log; exit 1; }
grep -v amdgpu $OUT/host_time_rb3.log | tail -3
