cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 200 python bench.py --part scan --no-cpu-baseline > gpurun_out/bs$i.log 2>&1 || exit 1
  python - "$i" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/bs{sys.argv[1]}.log").read().strip().splitlines()[-1])
r = d["retrieval"]["call_level"]
print(r["serial_us_per_call"], r["pipelined_us_per_batch"])
PY
done
