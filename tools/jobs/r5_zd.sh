#!/bin/bash
# round 5 job zd: the C2 step's split-K-capable GEMMs (tools/split_shapes.py) and the C2
# retrieval's batches in flight (tools/scan_depth.py)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 240 python -u tools/split_shapes.py > gpurun_out/r5_zd_split_shapes.txt 2>&1 || { tail -20 gpurun_out/r5_zd_split_shapes.txt; exit 1; }
grep -v Warning gpurun_out/r5_zd_split_shapes.txt | tail -30
timeout -k 10 240 python -u tools/scan_depth.py > gpurun_out/r5_zd_scan_depth.txt 2>&1 || { tail -20 gpurun_out/r5_zd_scan_depth.txt; exit 1; }
cat gpurun_out/r5_zd_scan_depth.txt
