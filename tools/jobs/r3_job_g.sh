# Fused InfoNCE + MX-fp8 + device corpus tests, MX GEMM variants, C2/C5 train legs, e2e main.py.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests/test_fp8_encoder_gpu.py tests/test_configs_gpu.py \
  tests/test_model_gpu.py tests/test_train_gpu.py tests/test_dist_gpu.py tests/test_main_gpu.py \
  tests/test_wordpiece.py -m gpu -q -rfE -s --timeout 300 --timeout-method thread > gpurun_out/pytest_g.log 2>&1
prc=$?
grep -E "passed|failed|^FAILED|BERT-base fp8|C5 fp8|fused|gemm_mx" gpurun_out/pytest_g.log | tail -40
[ $prc -eq 0 ] || [ $prc -eq 1 ] || exit $prc
V=information-retrieval-with-contrastive-learning_amd/irc_amd/lib/variants
for v in base mx_norederive noepi; do
  if [ $v = base ]; then L=; else L=$V/$v.so; fi
  IRC_LIB_PATH=$L timeout -k 10 200 python tools/gemm_bench.py --mx > gpurun_out/gemm_g_mx_$v.txt 2>&1 || exit 1
  echo "== $v"; grep -v amdgpu gpurun_out/gemm_g_mx_$v.txt
done
for part in train train_fp8; do
  timeout -k 10 400 python bench.py --part $part --no-cpu-baseline > gpurun_out/bench_g_$part.log 2>&1 || { tail -5 gpurun_out/bench_g_$part.log; exit 1; }
done
python - <<'PY'
import json
for part in ('train', 'train_fp8'):
    l=[x for x in open(f'gpurun_out/bench_g_{part}.log') if x.startswith('{')][-1]
    d=json.loads(l); t=d.get('train_fp8') if part=='train_fp8' else d
    r=t['roofline'] if part=='train_fp8' else d['roofline']
    print(part, d['value'], r['frac'], r['gemm_ms_per_step'])
PY
timeout -k 10 600 python tools/e2e_train.py --steps 40 > gpurun_out/e2e_g.log 2>&1 || { tail -5 gpurun_out/e2e_g.log; exit 1; }
grep -E "tokenizer|end-to-end|host time" gpurun_out/e2e_g.log
exit $prc
