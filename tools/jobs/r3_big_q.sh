# gemm_big_kernel (256 x 384 tile: QKV, out-proj, FFN2) decomposition and A/B builds.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
V=information-retrieval-with-contrastive-learning_amd/irc_amd/lib/variants
SH=qkv,attn_out+res,ffn2+res,ffn1+gelu
timeout -k 10 200 python tools/gemm_bench.py --only $SH > gpurun_out/big_base.txt 2>&1 || exit 1
for v in big_nodma big_noepi big_nostore big_spread big_rpre; do
  IRC_LIB_PATH=$V/$v.so timeout -k 10 200 python tools/gemm_bench.py --only $SH > gpurun_out/$v.txt 2>&1 || exit 1
done
timeout -k 10 200 python tools/gemm_bench.py --only $SH > gpurun_out/big_base2.txt 2>&1 || exit 1
for v in big_base big_nodma big_noepi big_nostore big_spread big_rpre big_base2; do echo "== $v"; grep -v amdgpu.ids gpurun_out/$v.txt; done
