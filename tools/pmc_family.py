"""Per-family HBM traffic of the trainable-BERT step's GEMMs: from a
`--pmc FETCH_SIZE` pass and a `--pmc WRITE_SIZE` pass of the same command, group the bf16
GEMM dispatches by kernel template (operand layouts = family) and grid size (= shape),
and print HBM bytes per dispatch, (2 * FETCH_SIZE + WRITE_SIZE) * 1024 as in
tools/pmc_summary.py (gfx950 FETCH_SIZE counts a 16-B/lane stream at half).

    python tools/pmc_family.py <fetch_dir> <write_dir> [--json out.json]

Families (gemm_pp_kernel<AK, BK, ...> / gemm_big_kernel / gemm_kernel): fwd = both operands
K-major (A [M][K], B [N][K]); dX = A K-major, B K-outer (dY . W); dW = both K-outer
(dY^T . X, split-K slabs + splitk_reduce_kernel).
"""
import argparse
import csv
import glob
import json
import os
import re
from collections import defaultdict

GEMM = re.compile(r"gemm_big_kernel<|gemm_kernel<|gemm_pp_kernel<|splitk_reduce_kernel")


def family(name):
    m = re.search(r"gemm_pp_kernel<(true|false), (true|false)", name)
    if m:
        a, b = m.groups()
        return {("true", "true"): "fwd (pp)", ("true", "false"): "dX (pp)",
                ("false", "false"): "dW (pp)", ("false", "true"): "A^T B^T (pp)"}[(a, b)]
    if "gemm_big_kernel" in name:
        return "fwd (big)"
    if "splitk_reduce" in name:
        return "dW split-K reduce"
    return "general"


def load(d, counter):
    out = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if r["Counter_Name"] != counter or not GEMM.search(r["Kernel_Name"]):
                    continue
                key = (f, r["Dispatch_Id"])
                v = out.setdefault(key, [r["Kernel_Name"], r.get("Grid_Size", "?"), 0.0])
                v[2] += float(r["Counter_Value"])
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    fe, wr = load(a.fetch_dir, "FETCH_SIZE"), load(a.write_dir, "WRITE_SIZE")
    agg = defaultdict(lambda: [0, 0.0, 0.0])
    for (_, _), (name, grid, v) in fe.items():
        k = (family(name), grid)
        agg[k][0] += 1
        agg[k][1] += v
    for (_, _), (name, grid, v) in wr.items():
        agg[(family(name), grid)][2] += v
    rows = []
    for (fam, grid), (n, f, w) in sorted(agg.items()):
        if n == 0:
            continue
        per = (2 * f + w) * 1024 / n
        rows.append({"family": fam, "grid": grid, "dispatches": n, "hbm_bytes_per_dispatch": per,
                     "read_bytes": 2 * f * 1024 / n, "write_bytes": w * 1024 / n})
        print(f"{fam:20s} grid={grid:>9s} n={n:4d}  HBM {per / 1e6:8.2f} MB/dispatch "
              f"(read {2 * f * 1.024e-3 / n:7.2f}, write {w * 1.024e-3 / n:7.2f})")
    if a.json:
        with open(a.json, "w") as fh:
            json.dump(rows, fh, indent=1)


if __name__ == "__main__":
    main()
