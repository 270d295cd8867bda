cd "$GRAFT_REPO_ROOT" || exit 1
L=$GRAFT_REPO_ROOT/information-retrieval-with-contrastive-learning_amd/irc_amd/lib/variants/stamps.so
IRC_LIB_PATH=$L timeout -k 10 120 python tools/dense_stats.py --q 1 16 64 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 120 python3 tools/scan_bench.py --reps 100 --q 1 16 32 64 2>&1 | grep -v amdgpu.ids || exit 1
