# C2 training step A/B: ping-pong GEMM one tile per workgroup vs the persistent
# dynamic-tile form (IRC_GEMM_PERSIST=1), alternating, three runs each.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2 3; do
  for m in 0 1; do
    IRC_GEMM_PERSIST=$m timeout -k 10 200 python bench.py --part train --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/pers_${m}_$r.log 2>&1 || exit 1
    python - gpurun_out/pers_${m}_$r.log $m <<'PY'
import json, sys
l = [x for x in open(sys.argv[1]) if x.startswith('{')][0]
d = json.loads(l)
print("persist", sys.argv[2], round(d["value"]), round(d["ms_per_step"], 3), round(d["roofline"]["frac"], 4))
PY
  done
done
