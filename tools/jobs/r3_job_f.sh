# MX-fp8 + device-corpus tests, big-kernel epilogue/DMA variants, fp8 bench, e2e main.py.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_fp8_encoder_gpu.py tests/test_wordpiece.py \
  tests/test_main_gpu.py "tests/test_configs_gpu.py::test_c5_fp8_step_loss_vs_fp32" -m gpu -q -rfE -s \
  --timeout 300 --timeout-method thread > gpurun_out/pytest_f.log 2>&1
prc=$?
grep -E "passed|failed|^FAILED|BERT-base fp8|C5 fp8" gpurun_out/pytest_f.log | tail -25
[ $prc -eq 0 ] || [ $prc -eq 1 ] || exit $prc
V=information-retrieval-with-contrastive-learning_amd/irc_amd/lib/variants
SH=qkv,attn_out+res,ffn2+res,lstm_xp_l0
for v in base spread rpre spread_rpre; do
  if [ $v = base ]; then L=; else L=$V/$v.so; fi
  IRC_LIB_PATH=$L timeout -k 10 200 python tools/gemm_bench.py --only $SH > gpurun_out/gemm_f_$v.txt 2>&1 || exit 1
  echo "== $v"; grep -v amdgpu gpurun_out/gemm_f_$v.txt
done
timeout -k 10 400 python bench.py --part train_fp8 --no-cpu-baseline > gpurun_out/bench_f_fp8.log 2>&1 || { tail -5 gpurun_out/bench_f_fp8.log; exit 1; }
python - <<'PY'
import json
l=[x for x in open('gpurun_out/bench_f_fp8.log') if x.startswith('{')][-1]
d=json.loads(l)['train_fp8']; print('train_fp8', d['pairs_per_s'], d['roofline']['frac'], d['roofline']['gemm_ms_per_step'])
PY
timeout -k 10 600 python tools/e2e_train.py --steps 40 > gpurun_out/e2e_f.log 2>&1 || { tail -5 gpurun_out/e2e_f.log; exit 1; }
grep -E "tokenizer|end-to-end|host time" gpurun_out/e2e_f.log
exit $prc
