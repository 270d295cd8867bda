# Refresh the C2 scan filter's PMC traffic (FETCH_SIZE and WRITE_SIZE passes) at HEAD.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc2
mkdir -p $OUT
cd /tmp || exit 1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 200 rocprofv3 --pmc $c --output-format csv -d $OUT/scan_c2_$c -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --part scan_c2 --steps 3 --warmup 1 --no-cpu-baseline \
    > $OUT/scan_c2_$c.log 2>&1 || { echo "pass $c failed"; exit 1; }
done
exit 0
