# Fused InfoNCE v2 (LDS-staged tiles) + MX epilogue (bit exponent, DPP quad max)
# tests; MX GEMM timing; C3 scan filter diagnostics; train legs; e2e (event-timed).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_configs_gpu.py tests/test_fp8_encoder_gpu.py \
  tests/test_model_gpu.py tests/test_dist_gpu.py tests/test_main_gpu.py tests/test_oracle_golden.py \
  -m gpu -q -rfE -s --timeout 300 --timeout-method thread > gpurun_out/pytest_h.log 2>&1
prc=$?
grep -E "passed|failed|^FAILED|C5 fp8|fused|Error" gpurun_out/pytest_h.log | tail -30
[ $prc -eq 0 ] || [ $prc -eq 1 ] || exit $prc
timeout -k 10 200 python tools/gemm_bench.py --mx > gpurun_out/gemm_h_mx.txt 2>&1 || exit 1
grep -v amdgpu gpurun_out/gemm_h_mx.txt
V=information-retrieval-with-contrastive-learning_amd/irc_amd/lib/variants
for v in base scan_dma scan_noepi scan_nocand; do
  if [ $v = base ]; then L=; else L=$V/$v.so; fi
  echo "== $v"
  IRC_LIB_PATH=$L timeout -k 10 200 python tools/scan_bench.py --n 250000 --q 1 16 64 256 --reps 30 > gpurun_out/scan_h_$v.txt 2>&1 || { tail -3 gpurun_out/scan_h_$v.txt; exit 1; }
  grep -v amdgpu gpurun_out/scan_h_$v.txt
done
IRC_LIB_PATH=$V/scan_stamps.so timeout -k 10 200 python tools/scan_blocks.py --n 250000 --q 1 16 64 > gpurun_out/scan_h_blocks.txt 2>&1 || { tail -3 gpurun_out/scan_h_blocks.txt; exit 1; }
grep -v amdgpu gpurun_out/scan_h_blocks.txt
for part in train train_fp8; do
  timeout -k 10 400 python bench.py --part $part --no-cpu-baseline > gpurun_out/bench_h_$part.log 2>&1 || { tail -5 gpurun_out/bench_h_$part.log; exit 1; }
done
python - <<'PY'
import json
for part in ('train', 'train_fp8'):
    l=[x for x in open(f'gpurun_out/bench_h_{part}.log') if x.startswith('{')][-1]
    d=json.loads(l); t=d.get('train_fp8') if part=='train_fp8' else d
    r=t['roofline'] if part=='train_fp8' else d['roofline']
    print(part, d['value'] if part=='train' else t['pairs_per_s'], r['frac'], r['gemm_ms_per_step'])
PY
timeout -k 10 600 python tools/e2e_train.py --steps 100 > gpurun_out/e2e_h.log 2>&1 || { tail -5 gpurun_out/e2e_h.log; exit 1; }
grep -E "tokenizer|end-to-end|host time" gpurun_out/e2e_h.log
exit $prc
