# Threshold-sample sweep of the C2 scan (IRC_SCAN_SAMPLE_DIV): whole-call and filter time per Q.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for d in 8 16 32 64 4; do
  IRC_SCAN_SAMPLE_DIV=$d timeout -k 10 120 python tools/scan_bench.py --q 64 256 1024 --reps 50 > gpurun_out/sdiv_$d.log 2>&1 || exit $?
done
exit 0
