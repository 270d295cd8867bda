# Round 4 job ak: main.py end to end -- what the 1.3 ms/step gap to the train leg is made of:
# DataLoader workers 6 vs 0, and sentences long enough that every batch pads to L = 64.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/r4ak
mkdir -p $OUT
for cfg in "--workers 6" "--workers 0" "--workers 6 --max-words 40"; do
  tag=$(echo $cfg | tr -d ' -')
  timeout -k 10 400 python tools/e2e_train.py --steps 80 $cfg > $OUT/e2e_$tag.log 2>&1 || { tail -20 $OUT/e2e_$tag.log; exit 1; }
  echo "== $cfg"; grep -E "end-to-end|host time" $OUT/e2e_$tag.log
done
