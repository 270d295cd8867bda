# Round 4 job an: heads-alone / BERT-alone / overlapped step on the closing code.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/r4an
mkdir -p $OUT
timeout -k 10 300 python tools/host_time.py --steps 30 > $OUT/host_time.log 2>&1 || { tail -20 $OUT/host_time.log; exit 1; }
grep -v amdgpu $OUT/host_time.log | tail -3
