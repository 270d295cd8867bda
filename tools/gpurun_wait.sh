#!/bin/bash
# Submit one gpurun command; when the pool has no box (status=transient: nothing ran,
# nothing charged), wait and submit it again, up to 12 times.  A call that ran is
# never re-submitted, whatever its result.
#   tools/gpurun_wait.sh <timeout_s> '<command>'
t=$1; shift
for i in $(seq 1 12); do
  out=$(/usr/local/graft/bin/gpurun --timeout "$t" -- "$@" 2>&1)
  echo "$out" | tail -60
  if echo "$out" | grep -q "status=transient"; then
    echo "[gpurun_wait] attempt $i: no box; waiting"
    sleep 150
    continue
  fi
  exit 0
done
exit 3
