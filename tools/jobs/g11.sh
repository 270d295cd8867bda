# LSTM recurrence family A/B inside the overlapped training step (bench --part train).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in coop mfma coop; do
  IRC_LSTM_RECURRENCE=$r timeout -k 10 200 python bench.py --part train --no-cpu-baseline > gpurun_out/lstm_$r.log 2>&1 || exit $?
  grep -o '"value": [0-9.]*' gpurun_out/lstm_$r.log | head -1
done
exit 0
