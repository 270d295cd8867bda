# Round 4 job ac: run-to-run reproducibility of the cluster LSTM backward, flag (R1) and
# tagged-granule (R2) hand-offs, against each other and the single-CU recurrence.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/r4ac
mkdir -p $OUT
timeout -k 10 300 python tools/lstm_coop_repro.py --n 8 > $OUT/repro.log 2>&1 || { tail -20 $OUT/repro.log; exit 1; }
grep -v amdgpu $OUT/repro.log
timeout -k 10 300 python tools/lstm_coop_repro.py --n 8 --b 40 --l 7 > $OUT/repro_small.log 2>&1 || { tail -20 $OUT/repro_small.log; exit 1; }
grep -v amdgpu $OUT/repro_small.log
