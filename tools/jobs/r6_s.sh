#!/bin/bash
# round 6 job s: the split forms' tail GEMMs under a grid cap (256 x 256 tiles on a few CUs
# beside the whole-wave chain, instead of the general kernel): parity tests, then main.py end
# to end (38% of its batches pad to L = 65-69 and split) with the cap against without it,
# interleaved twice.
# (Measured, then reverted: the tail grid cap and tools/e2e_train.py --tail-cap are gone; the
# logs are profiles/r06_s/.)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6_s
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_bert_split_gpu.py tests/test_gemm_gpu.py tests/test_model_gpu.py \
  tests/test_train_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
  for cap in 64 0; do
    timeout -k 10 400 python -u tools/e2e_train.py --steps 80 --tail-cap $cap > $O/e2e_cap${cap}_$rep.log 2>&1 \
      || { tail $O/e2e_cap${cap}_$rep.log; exit 1; }
    echo "cap $cap rep $rep $(grep end-to-end $O/e2e_cap${cap}_$rep.log)"
  done
done
