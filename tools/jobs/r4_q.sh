# Round 4 job q: the BERT-feature prefetch stream at high priority vs default (C2 step,
# interleaved on one box).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/r4q
mkdir -p $OUT
for r in 1 2 3; do
  for m in none bert_prefetch; do
    if [ $m = none ]; then unset IRC_HIGH_PRIORITY_STREAMS; else export IRC_HIGH_PRIORITY_STREAMS=$m; fi
    timeout -k 10 200 python bench.py --part train --steps 30 --warmup 5 --no-cpu-baseline > $OUT/train_${m}_$r.log 2>&1 || exit 1
    python3 - $OUT/train_${m}_$r.log $m <<'PY'
import json, sys
d = json.loads([x for x in open(sys.argv[1]) if x.startswith('{')][-1])
print("train high=%s" % sys.argv[2], round(d["value"]), round(d["ms_per_step"], 3))
PY
  done
done
