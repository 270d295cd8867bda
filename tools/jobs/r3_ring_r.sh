# gemm_big ring: bitwise test vs the 2-slot loop, GEMM tests, then the BERT-shape A/B and the C2 step A/B.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py tests/test_encoder_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ring_tests.log 2>&1 || { tail -30 gpurun_out/ring_tests.log; exit 1; }
tail -2 gpurun_out/ring_tests.log
SH=qkv,attn_out+res,ffn2+res,ffn1+gelu,ffn1+bias,square4k
for r in 1 2; do
  IRC_BIG_RING=1 timeout -k 10 200 python tools/gemm_bench.py --only $SH > gpurun_out/ring_on_$r.txt 2>&1 || exit 1
  IRC_BIG_RING=0 timeout -k 10 200 python tools/gemm_bench.py --only $SH > gpurun_out/ring_off_$r.txt 2>&1 || exit 1
done
# FFN1 (N = 3072) on the big-tile kernel instead of the ping-pong one
IRC_GEMM_PP=0 IRC_BIG_RING=1 timeout -k 10 200 python tools/gemm_bench.py --only ffn1+gelu,ffn1+bias > gpurun_out/ring_nopp_on.txt 2>&1 || exit 1
IRC_GEMM_PP=0 IRC_BIG_RING=0 timeout -k 10 200 python tools/gemm_bench.py --only ffn1+gelu,ffn1+bias > gpurun_out/ring_nopp_off.txt 2>&1 || exit 1
for f in ring_on_1 ring_off_1 ring_on_2 ring_off_2 ring_nopp_on ring_nopp_off; do echo "== $f"; grep -v amdgpu.ids gpurun_out/$f.txt; done
for r in 1 2; do
  for m in 1 0; do
    IRC_BIG_RING=$m timeout -k 10 200 python bench.py --part train --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/ring_train_${m}_$r.log 2>&1 || exit 1
    python - gpurun_out/ring_train_${m}_$r.log $m <<'PY'
import json, sys
l = [x for x in open(sys.argv[1]) if x.startswith('{')][0]
d = json.loads(l)
print("ring", sys.argv[2], round(d["value"]), round(d["ms_per_step"], 3), round(d["roofline"]["frac"], 4))
PY
  done
done
