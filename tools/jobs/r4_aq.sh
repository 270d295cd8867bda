# Round 4 job aq: cluster forward granule sweep without the s_sleep between passes
# (diagnostic build variants/nosleep.so) against the release build.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/r4aq
mkdir -p $OUT
V=$GRAFT_REPO_ROOT/information-retrieval-with-contrastive-learning_amd/irc_amd/lib/variants/nosleep.so
timeout -k 10 300 python tools/lstm_coop_repro.py --n 4 > $OUT/repro_rel.log 2>&1 || { tail -20 $OUT/repro_rel.log; exit 1; }
IRC_LIB_PATH=$V timeout -k 10 300 python tools/lstm_coop_repro.py --n 4 > $OUT/repro_late.log 2>&1 || { tail -20 $OUT/repro_late.log; exit 1; }
grep "tagged=0" $OUT/repro_rel.log $OUT/repro_late.log
for i in 1 2; do
  timeout -k 10 300 python tools/lstm_coop_bench.py --ab IRC_NONE=0 > $OUT/bench_rel$i.log 2>&1 || { tail -20 $OUT/bench_rel$i.log; exit 1; }
  echo "release $(grep 'round 1' $OUT/bench_rel$i.log)"
  IRC_LIB_PATH=$V timeout -k 10 300 python tools/lstm_coop_bench.py --ab IRC_NONE=0 > $OUT/bench_late$i.log 2>&1 || { tail -20 $OUT/bench_late$i.log; exit 1; }
  echo "nosleep $(grep 'round 1' $OUT/bench_late$i.log)"
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_lstm_mfma_gpu.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
