# Round 4 job t: the retrieval legs' pipelined rate fell 2.5x in run s (serial calls
# unchanged) -- the high-priority BERT-prefetch stream the train legs create is the suspect.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/r4t
mkdir -p $OUT
summ() {
python3 - $1 $2 <<'PY'
import json, sys
d = json.loads([x for x in open(sys.argv[1]) if x.startswith('{')][-1])
legs = d.get("legs", {})
print(sys.argv[2], "value", round(d["value"]), {k: v.get("queries_per_s", v.get("pairs_per_s")) for k, v in legs.items()})
PY
}
timeout -k 10 300 python bench.py --part scan > $OUT/scan_only.log 2>&1 || exit 1
summ $OUT/scan_only.log scan_only
IRC_HIGH_PRIORITY_STREAMS=none timeout -k 10 600 python bench.py > $OUT/all_none.log 2>&1 || exit 1
summ $OUT/all_none.log all_none
timeout -k 10 600 python bench.py > $OUT/all_default.log 2>&1 || exit 1
summ $OUT/all_default.log all_default
