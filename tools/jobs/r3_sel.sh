# Round-3 GPU job: selected -m gpu tests (no -x), then optional bench parts.
# usage: tools/jobs/r3_sel.sh TAG "pytest targets" [bench parts...]
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
tag=$1; targets=$2; shift 2
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest $targets -m gpu -q -rfE -s --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_$tag.log 2>&1
prc=$?
grep -E "passed|failed|FAILED|Error|BERT-base fp8|C5 fp8|Q=" gpurun_out/pytest_$tag.log | tail -30
[ $prc -eq 0 ] || [ $prc -eq 1 ] || exit $prc
for part in "$@"; do
  timeout -k 10 400 python bench.py --part $part --no-cpu-baseline > gpurun_out/bench_${tag}_$part.log 2>&1 || { tail -20 gpurun_out/bench_${tag}_$part.log; exit 1; }
  tail -c 600 gpurun_out/bench_${tag}_$part.log
done
exit $prc
