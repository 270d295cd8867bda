# select_dense phase stamps (diagnostic build) and kernel-trace times per Q on a C3-sized shard.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
V=$GRAFT_REPO_ROOT/information-retrieval-with-contrastive-learning_amd/irc_amd/lib/variants
IRC_LIB_PATH=$V/stamps.so timeout -k 10 200 python tools/dense_time.py > gpurun_out/dense_time.txt 2>&1 || { tail -20 gpurun_out/dense_time.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/dense_time.txt
cd /tmp
for q in 1 16 64; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_dense_$q -o run -- \
    python3 $GRAFT_REPO_ROOT/tools/dense_time.py --q $q > $GRAFT_REPO_ROOT/gpurun_out/prof_dense_$q.log 2>&1 || exit 1
done
for q in 1 16 64; do echo "== Q=$q"; f=$(find $GRAFT_REPO_ROOT/gpurun_out/prof_dense_$q -name '*kernel_stats.csv' | head -1); cut -d, -f1-5 "$f" | head -6; done
