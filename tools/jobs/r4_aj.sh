# Round 4 job aj (closing): cluster-LSTM reproducibility, the per-wave publish A/B, then the
# full GPU suite, smoke, the default bench line and the kernel-trace summaries
# (tools/jobs/r4_c.sh, TAG=aj).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/r4aj
mkdir -p $OUT
timeout -k 10 300 python tools/lstm_coop_repro.py --n 8 > $OUT/repro.log 2>&1 || { tail -20 $OUT/repro.log; exit 1; }
grep -v amdgpu $OUT/repro.log
timeout -k 10 300 python tools/lstm_coop_bench.py --ab IRC_LSTM_COOP_WAVE_PUBLISH=1,IRC_LSTM_COOP_WAVE_PUBLISH=0 > $OUT/lstm_wpub_ab.log 2>&1 || { tail -20 $OUT/lstm_wpub_ab.log; exit 1; }
grep round $OUT/lstm_wpub_ab.log
TAG=aj bash tools/jobs/r4_c.sh
