"""HBM traffic per GEMM shape against its algorithmic bytes (the
trainable-BERT step's GEMM families, fwd / dX / dW, one shape per family member).

tools/jobs/r4_h.sh runs `rocprofv3 --pmc FETCH_SIZE` and `--pmc WRITE_SIZE` passes of
`tools/gemm_bench.py --only <shape>` into <root>/<shape>_<COUNTER>/; this sums the
counter over the GEMM dispatches (the split-K reduce included), divides by the number of
GEMM calls, and prints HBM bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 as
tools/pmc_summary.py does (gfx950 FETCH_SIZE counts a 16-B/lane stream at half;
MI355X_MICROARCH.md, HBM / rocprofv3), next to the algorithmic bytes:
A + B + C (+ R read for residual / GELU' epilogues, + R written for the GELU-save
epilogue, + C read for fp32 accumulate).

    python tools/pmc_shapes.py <root> <shape> [<shape> ...] [--json out.json]
"""
import argparse
import csv
import glob
import json
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gemm_bench import SHAPES  # noqa: E402

GEMM = re.compile(r"gemm_big_kernel|gemm_kernel|gemm_pp_kernel|splitk_reduce_kernel")
MAIN = re.compile(r"gemm_big_kernel|gemm_kernel|gemm_pp_kernel")


def family(name, epi):
    if epi < 0:
        return "dW (A^T B, K-outer)"
    if epi in (4, 5) and "bert" in name:
        return "dX"
    return "fwd"


def alg_bytes(M, N, K, epi, name):
    if epi < 0:  # bf16 A [K][M], B [K][N]; fp32 C read + written (accumulate)
        return 2 * (M * K + N * K) + 8 * M * N
    out = 4 if name == "lstm_dx" or name.startswith("lstm_xp") else 2
    b = 2 * (M * K + N * K) + out * M * N
    if epi in (3, 4, 5):
        b += out * M * N
    if epi == 6:
        b += 2 * M * N
    return b


def load(d, counter):
    tot, calls = 0.0, set()
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if r["Counter_Name"] != counter or not GEMM.search(r["Kernel_Name"]):
                    continue
                tot += float(r["Counter_Value"])
                if MAIN.search(r["Kernel_Name"]):
                    calls.add((f, r["Dispatch_Id"]))
    return tot, len(calls)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("shapes", nargs="+")
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    table = {s[0]: s[1:] for s in SHAPES}
    rows = []
    print(f"{'shape':14s} {'family':20s} {'M':>6s} {'N':>6s} {'K':>6s}  {'alg MB':>8s} "
          f"{'HBM MB':>8s}  ratio")
    for s in a.shapes:
        M, N, K, epi = table[s]
        fe, n = load(os.path.join(a.root, f"{s}_FETCH_SIZE"), "FETCH_SIZE")
        wr, n2 = load(os.path.join(a.root, f"{s}_WRITE_SIZE"), "WRITE_SIZE")
        if n == 0 or n2 == 0:
            print(f"{s:14s} (no dispatches)")
            continue
        hbm = (2 * fe / n + wr / n2) * 1024
        alg = alg_bytes(M, N, K, epi, s)
        rows.append({"shape": s, "family": family(s, epi), "M": M, "N": N, "K": K, "epilogue": epi,
                     "alg_bytes": alg, "hbm_bytes": hbm, "ratio": hbm / alg,
                     "read_bytes": 2 * fe * 1024 / n, "write_bytes": wr * 1024 / n2})
        print(f"{s:14s} {family(s, epi):20s} {M:6d} {N:6d} {K:6d}  {alg / 1e6:8.1f} "
              f"{hbm / 1e6:8.1f}  {hbm / alg:5.2f}")
    if a.json:
        with open(a.json, "w") as fh:
            json.dump(rows, fh, indent=1)


if __name__ == "__main__":
    main()
