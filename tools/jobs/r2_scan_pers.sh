# Persistent scan filter (EPI_SCAN, bf16 + fp8): scan tests in modes 1 and 2 (mode 0 = the
# release default, covered by the full suite), then the retrieval bench legs per mode.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for m in 1 2; do
  IRC_GEMM_PERSIST=$m timeout -k 10 600 python -u -m pytest tests/test_scan_gpu.py tests/test_scan_fp8_gpu.py tests/test_configs_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread \
    > gpurun_out/pytest_scan_m$m.log 2>&1 || { tail -30 gpurun_out/pytest_scan_m$m.log; exit 1; }
  tail -1 gpurun_out/pytest_scan_m$m.log
done
for m in 0 1 2; do
  IRC_GEMM_PERSIST=$m timeout -k 10 400 python bench.py --part scan --no-cpu-baseline > gpurun_out/scan_m$m.log 2>&1 || { tail -20 gpurun_out/scan_m$m.log; exit 1; }
  echo mode $m; python - gpurun_out/scan_m$m.log <<'PY'
import json, sys
line = [l for l in open(sys.argv[1]) if l.startswith('{')][-1]
d = json.loads(line)
for k in ("retrieval", "retrieval_c4", "retrieval_fp8"):
    r = d.get(k) or {}
    c = r.get("call_level") or {}
    print(k, r.get("value"), "serial_us", c.get("serial_us_per_call"), "filter_frac", c.get("filter_hbm_frac"),
          "roof", (r.get("roofline") or {}).get("frac"))
PY
done
exit 0
