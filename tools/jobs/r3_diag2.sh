cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python tools/probe/mx_probe2.py > gpurun_out/mx_probe2.txt 2>&1 || { tail gpurun_out/mx_probe2.txt; exit 1; }
V=information-retrieval-with-contrastive-learning_amd/irc_amd/lib/variants
SH=qkv,attn_out+res,ffn1+gelu,ffn1+bias,ffn2+res,lstm_xp_l0,square4k
IRC_LIB_PATH=$V/noepi.so timeout -k 10 200 python tools/gemm_bench.py --only $SH > gpurun_out/gemm_noepi.txt 2>&1 || exit 1
grep -v amdgpu gpurun_out/gemm_noepi.txt
