# Round 4 job am: cluster LSTM backward with counted member flags (form 3: no producer-side
# barrier) against the workgroup flag form -- reproducibility, timing A/B, LSTM tests.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/r4am
mkdir -p $OUT
timeout -k 10 300 python tools/lstm_coop_repro.py --n 8 > $OUT/repro.log 2>&1 || { tail -20 $OUT/repro.log; exit 1; }
grep -v amdgpu $OUT/repro.log
timeout -k 10 300 python tools/lstm_coop_bench.py --ab IRC_LSTM_COOP_BWD_TAGGED=0,IRC_LSTM_COOP_BWD_TAGGED=3 > $OUT/lstm_bwd_ab.log 2>&1 || { tail -20 $OUT/lstm_bwd_ab.log; exit 1; }
grep round $OUT/lstm_bwd_ab.log
IRC_LSTM_COOP_BWD_TAGGED=3 timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_lstm_mfma_gpu.py tests/test_train_gpu.py > $OUT/tests3.log 2>&1 || { tail -30 $OUT/tests3.log; exit 1; }
tail -1 $OUT/tests3.log
