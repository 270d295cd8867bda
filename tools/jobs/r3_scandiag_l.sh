# Scan filter decomposition on the C3 shard (250k x 768 bf16, beyond the Infinity Cache):
# base, corpus stream only, + MFMAs, + exchange (no epilogue).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
V=information-retrieval-with-contrastive-learning_amd/irc_amd/lib/variants
timeout -k 10 150 python tools/scan_bench.py --n 250000 --q 1 16 64 256 > gpurun_out/scan_base.txt 2>&1 || exit 1
for v in scan_dmaonly scan_mfmaonly scan_noepi; do
  IRC_LIB_PATH=$V/$v.so timeout -k 10 150 python tools/scan_bench.py --n 250000 --q 1 16 64 --reps 10 > gpurun_out/$v.txt 2>&1 || exit 1
done
for v in scan_base scan_dmaonly scan_mfmaonly scan_noepi; do echo "== $v"; grep -v amdgpu.ids gpurun_out/$v.txt; done
