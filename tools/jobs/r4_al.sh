# Round 4 job al: main.py end to end with the pinned staging ring for the micro-batch indices
# against the per-call pin_memory() form, interleaved; the device-corpus test.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/r4al
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_wordpiece.py tests/test_main_gpu.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for r in 0 1 0 1; do
  IRC_CORPUS_PIN_RING=$r timeout -k 10 400 python tools/e2e_train.py --steps 80 > $OUT/e2e_ring$r.log 2>&1 || { tail -20 $OUT/e2e_ring$r.log; exit 1; }
  echo "ring=$r $(grep end-to-end $OUT/e2e_ring$r.log)"
done
