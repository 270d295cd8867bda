# Round 4 job ai: cluster forward with per-wave publish (no barrier between the cell update
# and the hand-off) against the workgroup publish -- bit identity, latency, tests, train leg.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/r4ai
mkdir -p $OUT
timeout -k 10 300 python tools/lstm_coop_bench.py --ab IRC_LSTM_COOP_WAVE_PUBLISH=0,IRC_LSTM_COOP_WAVE_PUBLISH=1 > $OUT/lstm_wpub_ab.log 2>&1 || { tail -20 $OUT/lstm_wpub_ab.log; exit 1; }
grep round $OUT/lstm_wpub_ab.log
timeout -k 10 300 python tools/lstm_coop_bench.py --b 40 --l 7 --iters 5 --ab IRC_LSTM_COOP_WAVE_PUBLISH=0,IRC_LSTM_COOP_WAVE_PUBLISH=1 > $OUT/lstm_wpub_small.log 2>&1 || { tail -20 $OUT/lstm_wpub_small.log; exit 1; }
grep round $OUT/lstm_wpub_small.log
IRC_LSTM_COOP_WAVE_PUBLISH=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_lstm_mfma_gpu.py tests/test_model_gpu.py tests/test_train_gpu.py > $OUT/tests_wpub.log 2>&1 \
  || { tail -30 $OUT/tests_wpub.log; exit 1; }
tail -1 $OUT/tests_wpub.log
for r in 0 1 0 1; do
IRC_LSTM_COOP_WAVE_PUBLISH=$r timeout -k 10 400 python bench.py --part train > $OUT/bench_train_w$r.log 2>&1 || { tail -20 $OUT/bench_train_w$r.log; exit 1; }
echo "wpub=$r $(grep '^{' $OUT/bench_train_w$r.log | tail -1 | cut -c90-150)"
done
