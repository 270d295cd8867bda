# Kernel trace of the training legs alone (bf16 frozen, fp8 frozen): per-kernel by grid.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
cd /tmp
for part in train train_fp8; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/prof_$part -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --part $part --no-cpu-baseline --steps 10 \
    > $GRAFT_REPO_ROOT/gpurun_out/prof_$part.log 2>&1 || exit 1
done
exit 0
