cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for cfg in "" "IRC_SCAN_PP=0" "IRC_SCAN_SAMPLE_DIV=8" "IRC_SCAN_SAMPLE_DIV=32"; do
  echo "== $cfg"
  env $cfg timeout -k 10 120 python tools/scan_bench.py --q 1 64 128 192 256 --reps 30 2>&1 | grep -v amdgpu.ids || exit 1
done
