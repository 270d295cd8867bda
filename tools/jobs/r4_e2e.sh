# Round 4: end-to-end training through main.py -> src.train (device corpus, GPU WordPiece,
# BERT prefetch, heads) at the C2 shapes, with the round-4 kernels.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/r4e2e
mkdir -p $OUT
timeout -k 10 600 python tools/e2e_train.py --steps 40 > $OUT/e2e.log 2>&1 || { tail -20 $OUT/e2e.log; exit 1; }
grep -v amdgpu $OUT/e2e.log | tail -12
