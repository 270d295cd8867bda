cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python tools/torch_gemm_ref.py > gpurun_out/torchgemm.log 2>&1 || exit $?
for k in 10 100 400; do
  (cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/prof_sk$k" -o run -- python3 "$GRAFT_REPO_ROOT/tools/scan_bench.py" --q 1 256 --k $k > "$GRAFT_REPO_ROOT/gpurun_out/sk$k.log" 2>&1) || exit $?
done
exit 0
