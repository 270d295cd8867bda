# Attention at any L <= 128 on MFMA (+ MX output staged through LDS), fused NCE
# combine/reduce, then the encoder split, NCE kernels, e2e and the train legs.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gemm_gpu.py tests/test_attention_gpu.py tests/test_fp8_encoder_gpu.py \
  tests/test_configs_gpu.py tests/test_model_gpu.py tests/test_train_gpu.py tests/test_main_gpu.py \
  tests/test_oracle_golden.py -m gpu -q -rfE -s --timeout 300 --timeout-method thread > gpurun_out/pytest_j.log 2>&1
prc=$?
grep -E "passed|failed|^FAILED|C5 fp8|fused|Error" gpurun_out/pytest_j.log | tail -30
[ $prc -eq 0 ] || [ $prc -eq 1 ] || exit $prc
V=information-retrieval-with-contrastive-learning_amd/irc_amd/lib/variants
for v in base g1off; do
  if [ $v = base ]; then L=; else L=$V/$v.so; fi
  echo "== gemm $v"
  IRC_LIB_PATH=$L timeout -k 10 200 python tools/gemm_bench.py --only qkv,attn_out+res,ffn1+gelu,ffn2+res,square4k > gpurun_out/gemm_j_$v.txt 2>&1 || { tail -3 gpurun_out/gemm_j_$v.txt; exit 1; }
  IRC_LIB_PATH=$L timeout -k 10 200 python tools/gemm_bench.py --mx >> gpurun_out/gemm_j_$v.txt 2>&1 || { tail -3 gpurun_out/gemm_j_$v.txt; exit 1; }
  grep -v amdgpu gpurun_out/gemm_j_$v.txt
done
timeout -k 10 200 python tools/nce_bench.py > gpurun_out/nce_j.txt 2>&1 || { tail -3 gpurun_out/nce_j.txt; exit 1; }
grep -v amdgpu gpurun_out/nce_j.txt
timeout -k 10 300 python tools/encode_bench.py > gpurun_out/encode_j.txt 2>&1 || { tail -3 gpurun_out/encode_j.txt; exit 1; }
grep -v amdgpu gpurun_out/encode_j.txt
timeout -k 10 600 python tools/e2e_train.py --steps 100 > gpurun_out/e2e_j.log 2>&1 || { tail -5 gpurun_out/e2e_j.log; exit 1; }
grep -E "tokenizer|end-to-end|host time" gpurun_out/e2e_j.log
for part in train train_fp8; do
  timeout -k 10 400 python bench.py --part $part --no-cpu-baseline > gpurun_out/bench_j_$part.log 2>&1 || { tail -5 gpurun_out/bench_j_$part.log; exit 1; }
done
python - <<'PY'
import json
for part in ('train', 'train_fp8'):
    l=[x for x in open(f'gpurun_out/bench_j_{part}.log') if x.startswith('{')][-1]
    d=json.loads(l); t=d.get('train_fp8') if part=='train_fp8' else d
    r=t['roofline'] if part=='train_fp8' else d['roofline']
    print(part, d['value'] if part=='train' else t['pairs_per_s'], r['frac'], r['gemm_ms_per_step'])
PY
exit $prc
