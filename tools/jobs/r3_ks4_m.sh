# Four-k-slice single-pass scan: parity tests with it on and off, then the C3 / C2 Q sweep A/B.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
IRC_SCAN_LTOP_KS4=1 timeout -k 10 300 python -u -m pytest tests/test_scan_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ks4_tests_on.log 2>&1 || { tail -30 gpurun_out/ks4_tests_on.log; exit 1; }
tail -2 gpurun_out/ks4_tests_on.log
timeout -k 10 300 python -u -m pytest tests/test_scan_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ks4_tests_off.log 2>&1 || { tail -30 gpurun_out/ks4_tests_off.log; exit 1; }
tail -2 gpurun_out/ks4_tests_off.log
for n in 250000 100000; do
  IRC_SCAN_LTOP_KS4=1 timeout -k 10 150 python tools/scan_bench.py --n $n --q 1 16 32 33 64 > gpurun_out/ks4_on_$n.txt 2>&1 || exit 1
  timeout -k 10 150 python tools/scan_bench.py --n $n --q 1 16 32 33 64 > gpurun_out/ks4_off_$n.txt 2>&1 || exit 1
done
for f in ks4_on_250000 ks4_off_250000 ks4_on_100000 ks4_off_100000; do echo "== $f"; grep -v amdgpu.ids gpurun_out/$f.txt; done
