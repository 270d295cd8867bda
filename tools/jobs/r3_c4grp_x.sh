# C4 leg (BERT-large GEMMs on the 256x256 ping-pong kernel): grouped output-tile order A/B.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do
  for gm in 0 4 8 16; do
    IRC_GEMM_GROUP_M=$gm timeout -k 10 200 python bench.py --part train_c4 --steps 12 --warmup 3 --no-cpu-baseline > gpurun_out/c4grp_${gm}_$r.log 2>&1 || { tail -20 gpurun_out/c4grp_${gm}_$r.log; exit 1; }
    python - gpurun_out/c4grp_${gm}_$r.log $gm <<'PY'
import json, sys
d = json.loads([x for x in open(sys.argv[1]) if x.startswith('{')][0])
t = d.get("train_c4") or d
print("group_m", sys.argv[2], round(t.get("pairs_per_s", d["value"])), round(d["ms_per_step"], 3),
      round(d["roofline"]["frac"], 4), round(d["roofline"]["gemm_ms_per_step"], 3))
PY
  done
done
