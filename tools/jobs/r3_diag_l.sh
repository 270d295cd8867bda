# GEMM time decomposition on the BERT shapes at HEAD (diagnostic builds of gemm_pp.hip):
# base, main loop without the next-tile DMA, main loop only, epilogue without C stores.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
V=information-retrieval-with-contrastive-learning_amd/irc_amd/lib/variants
SH=qkv,attn_out+res,ffn1+gelu,ffn1+bias,ffn2+res,lstm_xp_l0,square4k
timeout -k 10 200 python tools/gemm_bench.py --only $SH > gpurun_out/gemm_base.txt 2>&1 || exit 1
timeout -k 10 200 python tools/gemm_bench.py --mx > gpurun_out/gemm_mx_base.txt 2>&1 || exit 1
for v in nodma noepi nostore; do
  IRC_LIB_PATH=$V/$v.so timeout -k 10 200 python tools/gemm_bench.py --only $SH > gpurun_out/gemm_$v.txt 2>&1 || exit 1
  IRC_LIB_PATH=$V/$v.so timeout -k 10 200 python tools/gemm_bench.py --mx > gpurun_out/gemm_mx_$v.txt 2>&1 || exit 1
done
for v in base nodma noepi nostore; do echo "== $v"; grep -v amdgpu.ids gpurun_out/gemm_$v.txt; grep -v amdgpu.ids gpurun_out/gemm_mx_$v.txt; done
