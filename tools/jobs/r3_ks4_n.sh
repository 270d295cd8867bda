cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for c in "7 20000 1024 200 5" "40 25000 1024 64 0" "7 20000 768 200 5" "1 50011 768 100 0"; do
  for ks in 1 0; do
    IRC_SCAN_LTOP_KS4=$ks timeout -k 10 120 python tools/diag/ks4_case.py $c >> gpurun_out/ks4_diag.txt 2>&1 || exit 1
  done
  IRC_SCAN_LTOP=0 timeout -k 10 120 python tools/diag/ks4_case.py $c >> gpurun_out/ks4_diag.txt 2>&1 || exit 1
done
grep -v amdgpu.ids gpurun_out/ks4_diag.txt
