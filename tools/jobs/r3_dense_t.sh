# select_dense after the one-atomic collect and the vector rank: scan parity tests, phase
# stamps (diagnostic build), then the scan bench part (C2 / C3 Q sweeps).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_scan_gpu.py tests/test_scan_fp8_gpu.py tests/test_configs_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/dense_tests.log 2>&1 || { tail -30 gpurun_out/dense_tests.log; exit 1; }
tail -2 gpurun_out/dense_tests.log
V=$GRAFT_REPO_ROOT/information-retrieval-with-contrastive-learning_amd/irc_amd/lib/variants
IRC_LIB_PATH=$V/stamps.so timeout -k 10 200 python tools/dense_time.py > gpurun_out/dense_time4.txt 2>&1 || { tail -20 gpurun_out/dense_time4.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/dense_time4.txt
timeout -k 10 400 python bench.py --part scan --no-cpu-baseline > gpurun_out/dense_scan4.log 2>&1 || { tail -20 gpurun_out/dense_scan4.log; exit 1; }
python tools/sweep_print.py gpurun_out/dense_scan4.log
timeout -k 10 300 python bench.py --part train_c4 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/c4_check.log 2>&1 || { tail -20 gpurun_out/c4_check.log; exit 1; }
python - gpurun_out/c4_check.log <<'PY'
import json, sys
d = json.loads([x for x in open(sys.argv[1]) if x.startswith('{')][0])
r = d["roofline"]
print("train_c4", round(d["value"]), r["frac"], r["traffic"], r.get("traffic_over_alg"), r.get("traffic_source"))
PY
