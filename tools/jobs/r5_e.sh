#!/bin/bash
# round 5 job e: isolate the end-to-end gap (tools/e2e_probe.py)
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u tools/e2e_probe.py --steps 40 > gpurun_out/r5_e_probe.log 2>&1
rc=$?
grep -E "ms/step|Error|error" gpurun_out/r5_e_probe.log | tail -20
exit $rc
