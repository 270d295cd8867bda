"""One scan_topk case vs the oracle (diagnostic): prints mismatching rows, the
rescan counters, and where the missing docs sit (worker / tile row)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "information-retrieval-with-contrastive-learning_amd"))
from irc_amd import retrieval  # noqa: E402
from oracle import irc_oracle as O  # noqa: E402

Q, N, D, k, off = (int(x) for x in sys.argv[1:6])
rng = np.random.default_rng(Q * 7 + N)
q = rng.integers(-3, 4, (Q, D)).astype(np.float32) / 128  # tests/test_scan_gpu.py _grid(rng, shape, 3)
d = rng.integers(-3, 4, (N, D)).astype(np.float32) / 128
dev = torch.device("cuda:0")
retrieval.rescan_stats(reset=True)
s, i = retrieval.scan_topk(torch.from_numpy(q).to(dev), torch.from_numpy(d).to(dev), k, off)
nq, nw = retrieval.rescan_stats(reset=True)
ri, rs = O.scan_topk(q, d, k, doc_offset=off)
i, s = i.cpu().numpy(), s.cpu().numpy()
bad = [r for r in range(Q) if not np.array_equal(i[r], ri[r])]
print(f"env KS4={os.environ.get('IRC_SCAN_LTOP_KS4')} LTOP={os.environ.get('IRC_SCAN_LTOP')}: "
      f"rescans {nq} queries / {nw} workers; bad rows {bad}")
for r in bad[:3]:
    miss = sorted(set(ri[r]) - set(i[r]))
    extra = sorted(set(i[r]) - set(ri[r]))
    full = d @ q[r]
    print(" row", r, "kth oracle", rs[r, -1], "missing", [(m, float(full[m - off]), (m - off) // 32, (m - off) % 32) for m in miss][:8],
          "extra", [(m, float(full[m - off]), float(s[r][list(i[r]).index(m)])) for m in extra][:8])
    # scores returned vs the true scores of the returned docs
    wrong = [(int(m), float(sc), float(full[m - off])) for m, sc in zip(i[r], s[r]) if sc != full[m - off]]
    print("   returned docs with wrong scores:", wrong[:6])
