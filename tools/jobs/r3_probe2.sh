cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 120 python tools/probe/mx_probe2.py > gpurun_out/mx_probe2.txt 2>&1 || { tail gpurun_out/mx_probe2.txt; exit 1; }
grep -c lane gpurun_out/mx_probe2.txt
