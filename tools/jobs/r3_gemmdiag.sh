# MX lane-map probe + GEMM time decomposition (diagnostic builds) on the BERT shapes.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python tools/probe/mx_probe.py > gpurun_out/mx_probe.txt 2>&1 || { tail gpurun_out/mx_probe.txt; exit 1; }
V=information-retrieval-with-contrastive-learning_amd/irc_amd/lib/variants
SH=qkv,attn_out+res,ffn1+gelu,ffn1+bias,ffn2+res,lstm_xp_l0,square4k
timeout -k 10 200 python tools/gemm_bench.py --only $SH > gpurun_out/gemm_base.txt 2>&1 || exit 1
for v in nodma noepi nostore; do
  IRC_LIB_PATH=$V/$v.so timeout -k 10 200 python tools/gemm_bench.py --only $SH > gpurun_out/gemm_$v.txt 2>&1 || exit 1
done
IRC_LIB_PATH=$V/noopsel.so timeout -k 10 300 python -m pytest tests/test_fp8_encoder_gpu.py -m gpu -q -k "gemm_mx_vs" --timeout 120 > gpurun_out/pytest_noopsel.txt 2>&1
tail -3 gpurun_out/pytest_noopsel.txt
head -40 gpurun_out/mx_probe.txt
for v in base nodma noepi nostore; do echo "== $v"; grep -v amdgpu.ids gpurun_out/gemm_$v.txt; done
