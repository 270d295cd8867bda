# Round 4 job n: per-K-tile phase stamps of the big-tile 16x16x32 main loop (diagnostic
# build) on the BERT shapes, and the MX-fp8 GEMMs' current times.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/r4n
mkdir -p $OUT
V=$GRAFT_REPO_ROOT/information-retrieval-with-contrastive-learning_amd/irc_amd/lib/variants/bigstamps.so
for s in ffn2 qkv out ffn1; do
  IRC_LIB_PATH=$V timeout -k 10 120 python tools/big_stamps.py --shape $s > $OUT/stamps_$s.txt 2>&1 || { tail -5 $OUT/stamps_$s.txt; exit 1; }
  grep -v amdgpu $OUT/stamps_$s.txt
done
timeout -k 10 200 python tools/gemm_bench.py --mx > $OUT/mx.txt 2>&1 || exit 1
grep -v amdgpu $OUT/mx.txt
