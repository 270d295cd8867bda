# GEMM kernel choice for the BERT shapes: ping-pong (default) vs big-tile / general kernels.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python tools/gemm_bench.py --iters 30 > gpurun_out/gemm_pp_on.log 2>&1 || exit $?
IRC_GEMM_PP=0 timeout -k 10 120 python tools/gemm_bench.py --iters 30 > gpurun_out/gemm_pp_off.log 2>&1 || exit $?
exit 0
