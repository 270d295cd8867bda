# Round 4 job ad: after padding the inline-asm store hazard -- reproducibility of both
# backward hand-offs, their timing A/B, forward sentinel A/B, LSTM tests, heads-alone step.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/r4ad
mkdir -p $OUT
timeout -k 10 300 python tools/lstm_coop_repro.py --n 8 > $OUT/repro.log 2>&1 || { tail -20 $OUT/repro.log; exit 1; }
grep -v amdgpu $OUT/repro.log
timeout -k 10 300 python tools/lstm_coop_bench.py --ab IRC_LSTM_COOP_BWD_TAGGED=0,IRC_LSTM_COOP_BWD_TAGGED=1 > $OUT/lstm_bwd_ab.log 2>&1 || { tail -20 $OUT/lstm_bwd_ab.log; exit 1; }
grep round $OUT/lstm_bwd_ab.log
timeout -k 10 300 python tools/lstm_coop_bench.py --ab IRC_LSTM_COOP_SENTINELS=1,IRC_LSTM_COOP_SENTINELS=0 > $OUT/lstm_fwd_ab.log 2>&1 || { tail -20 $OUT/lstm_fwd_ab.log; exit 1; }
grep round $OUT/lstm_fwd_ab.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_lstm_mfma_gpu.py tests/test_model_gpu.py tests/test_train_gpu.py > $OUT/tests.log 2>&1 \
  || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 300 python tools/host_time.py --steps 30 > $OUT/host_time.log 2>&1 || { tail -20 $OUT/host_time.log; exit 1; }
grep -v amdgpu $OUT/host_time.log | tail -3
