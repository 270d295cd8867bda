cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
export IRC_SCAN_LTOP_KS4=1
mkdir -p gpurun_out
V=information-retrieval-with-contrastive-learning_amd/irc_amd/lib/variants
for c in "7 20000 1024 200 5" "1 50011 768 100 0" "33 40000 768 100 2"; do
  for rep in 1 2; do
    timeout -k 10 120 python tools/diag/ks4_case.py $c >> gpurun_out/ks4_diag2.txt 2>&1 || exit 1
    IRC_LIB_PATH=$V/xnowait.so timeout -k 10 120 python tools/diag/ks4_case.py $c >> gpurun_out/ks4_diag2.txt 2>&1 || exit 1
  done
done
grep -v amdgpu.ids gpurun_out/ks4_diag2.txt
