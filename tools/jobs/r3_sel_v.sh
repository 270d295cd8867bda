# select_fast with the threads' lower bound, one-atomic collect and vector rank: scan parity
# tests, then the scan bench part (C2 / C3 / C5 Q sweeps).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_scan_gpu.py tests/test_scan_fp8_gpu.py tests/test_configs_gpu.py tests/test_predict_gpu.py tests/test_dist_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/sel_tests.log 2>&1 || { tail -30 gpurun_out/sel_tests.log; exit 1; }
tail -2 gpurun_out/sel_tests.log
timeout -k 10 400 python bench.py --part scan --no-cpu-baseline > gpurun_out/sel_scan.log 2>&1 || { tail -20 gpurun_out/sel_scan.log; exit 1; }
python tools/sweep_print.py gpurun_out/sel_scan.log
python - gpurun_out/sel_scan.log <<'PY'
import json, sys
d = json.loads([x for x in open(sys.argv[1]) if x.startswith('{')][0])
for k in ("retrieval", "retrieval_c3", "retrieval_c4", "retrieval_fp8"):
    v = d.get(k) or {}
    print(k, round(v.get("value", 0)), "q/s", v.get("call_level", {}).get("serial_us_per_call"))
PY
