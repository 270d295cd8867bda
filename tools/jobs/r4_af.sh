# Round 4 job af (closing): cluster-LSTM backward forms (repro + timing A/B: workgroup flag
# vs per-wave flags), then the full GPU suite, smoke, the default bench line and the
# kernel-trace summaries (tools/jobs/r4_c.sh, TAG=af).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/r4af
mkdir -p $OUT
timeout -k 10 300 python tools/lstm_coop_repro.py --n 8 > $OUT/repro.log 2>&1 || { tail -20 $OUT/repro.log; exit 1; }
grep -v amdgpu $OUT/repro.log
timeout -k 10 300 python tools/lstm_coop_bench.py --ab IRC_LSTM_COOP_BWD_TAGGED=0,IRC_LSTM_COOP_BWD_TAGGED=2 > $OUT/lstm_bwd_ab.log 2>&1 || { tail -20 $OUT/lstm_bwd_ab.log; exit 1; }
grep round $OUT/lstm_bwd_ab.log
TAG=af bash tools/jobs/r4_c.sh
