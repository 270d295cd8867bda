# Scan: early DMA issue (exactness tests + C3 A/B + per-block timing); fused NCE
# kernel timing; frozen encoder bf16 vs MX-fp8 split; e2e main.py (event-timed).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_scan_gpu.py tests/test_configs_gpu.py tests/test_scan_fp8_gpu.py \
  -m gpu -q -rfE -s --timeout 300 --timeout-method thread > gpurun_out/pytest_i.log 2>&1
prc=$?
grep -E "passed|failed|^FAILED|Error" gpurun_out/pytest_i.log | tail -30
[ $prc -eq 0 ] || [ $prc -eq 1 ] || exit $prc
V=information-retrieval-with-contrastive-learning_amd/irc_amd/lib/variants
for v in base scan_early0 scan_dma scan_dma0; do
  if [ $v = base ]; then L=; else L=$V/$v.so; fi
  echo "== $v"
  IRC_LIB_PATH=$L timeout -k 10 200 python tools/scan_bench.py --n 250000 --q 1 16 64 256 --reps 30 > gpurun_out/scan_i_$v.txt 2>&1 || { tail -3 gpurun_out/scan_i_$v.txt; exit 1; }
  grep -v amdgpu gpurun_out/scan_i_$v.txt
done
IRC_LIB_PATH=$V/scan_stamps.so timeout -k 10 200 python tools/scan_blocks.py --n 250000 --q 1 16 64 > gpurun_out/scan_i_blocks.txt 2>&1 || { tail -3 gpurun_out/scan_i_blocks.txt; exit 1; }
grep -v amdgpu gpurun_out/scan_i_blocks.txt
timeout -k 10 200 python tools/nce_bench.py > gpurun_out/nce_i.txt 2>&1 || { tail -3 gpurun_out/nce_i.txt; exit 1; }
grep -v amdgpu gpurun_out/nce_i.txt
timeout -k 10 300 python tools/encode_bench.py > gpurun_out/encode_i.txt 2>&1 || { tail -3 gpurun_out/encode_i.txt; exit 1; }
grep -v amdgpu gpurun_out/encode_i.txt
timeout -k 10 600 python tools/e2e_train.py --steps 100 > gpurun_out/e2e_i.log 2>&1 || { tail -5 gpurun_out/e2e_i.log; exit 1; }
grep -E "tokenizer|end-to-end|host time" gpurun_out/e2e_i.log
exit $prc
