"""HBM bytes per launch from rocprofv3 --pmc passes -> profiles/pmc_<tag>.json.

Usage: python tools/pmc_summary.py <fetch_pass_dir> <write_pass_dir> <kernel_regex> <tag>
                                   [--grid N] [--note TEXT]

`fetch_pass_dir` holds a `--pmc FETCH_SIZE` run and `write_pass_dir` a `--pmc WRITE_SIZE`
run of the same command (the two cannot share a pass: FETCH_SIZE takes 3 of the 4 TCC
counters, WRITE_SIZE 2). Units and the gfx950 correction follow
/opt/skills/guides/MI355X_MICROARCH.md (HBM section): both counters are in KiB, and on gfx950
FETCH_SIZE reports half the bytes of a wide (16 B/lane) coalesced stream, so the read side is
doubled; WRITE_SIZE is exact for 16-B/lane stores and fp32 atomics.

    hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024     (per dispatch)

bench.py reads `hbm_bytes_per_launch` into its roofline `traffic` field.
"""
import argparse
import csv
import glob
import json
import os
import re


def _per_dispatch(d, counter, rx, grid):
    out = {}
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if r["Counter_Name"] != counter or not rx.search(r["Kernel_Name"]):
                    continue
                if grid is not None and int(r.get("Grid_Size", -1)) != grid:
                    continue
                key = (f, r["Dispatch_Id"])
                out[key] = out.get(key, 0.0) + float(r["Counter_Value"])
    return out, files


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("kernel_regex")
    ap.add_argument("tag")
    ap.add_argument("--grid", type=int, default=None)
    ap.add_argument("--note", default="")
    ap.add_argument("--out", default=os.path.join(os.path.dirname(__file__), "..", "profiles"))
    a = ap.parse_args()
    rx = re.compile(a.kernel_regex)
    fetch, _ = _per_dispatch(a.fetch_dir, "FETCH_SIZE", rx, a.grid)
    write, _ = _per_dispatch(a.write_dir, "WRITE_SIZE", rx, a.grid)
    if not fetch or not write:
        raise SystemExit(f"no dispatches matched {a.kernel_regex!r} (grid={a.grid})")
    f_kib = sum(fetch.values()) / len(fetch)
    w_kib = sum(write.values()) / len(write)
    res = {
        "tag": a.tag,
        "kernel_regex": a.kernel_regex,
        "grid": a.grid,
        "dispatches_fetch_pass": len(fetch),
        "dispatches_write_pass": len(write),
        "fetch_size_kib_per_launch_raw": f_kib,
        "write_size_kib_per_launch": w_kib,
        "read_bytes_per_launch": 2 * f_kib * 1024,
        "write_bytes_per_launch": w_kib * 1024,
        "hbm_bytes_per_launch": (2 * f_kib + w_kib) * 1024,
        "formula": "(2*FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950: FETCH_SIZE reads half of a "
                   "16-B/lane stream; KiB units)",
        "note": a.note,
    }
    os.makedirs(a.out, exist_ok=True)
    p = os.path.join(a.out, f"pmc_{a.tag}.json")
    with open(p, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
