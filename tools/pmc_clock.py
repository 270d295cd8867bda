"""Effective clock of the GEMM launches of a `tools/gemm_bench.py` run profiled with
`rocprofv3 --pmc GRBM_GUI_ACTIVE` (MI355X_MICROARCH.md, DVFS give-back: clock ~=
GRBM_GUI_ACTIVE / 8 / kernel wall time; rocprofv3 sums the counter over the 8 XCDs).

    python tools/pmc_clock.py <pmc_dir> <gemm_bench_log>

Pairs each shape line of the log (us per launch) with the mean GRBM_GUI_ACTIVE of that
run's GEMM dispatches (one shape per run), and prints the clock in GHz.
"""
import csv
import glob
import os
import re
import sys

GEMM = re.compile(r"gemm_big_kernel|gemm_kernel|gemm_pp_kernel|qkv_attn_kernel")


def main():
    d, log = sys.argv[1], sys.argv[2]
    vals = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if r["Counter_Name"] == "GRBM_GUI_ACTIVE" and GEMM.search(r["Kernel_Name"]):
                    vals.append(float(r["Counter_Value"]))
    us = [float(m.group(1)) for m in re.finditer(r"([0-9.]+) us", open(log).read())]
    if not vals or not us:
        print("no data")
        return
    g = sum(vals) / len(vals)
    t = sum(us) / len(us)
    print(f"{os.path.basename(d)}: GRBM_GUI_ACTIVE {g:.0f} per dispatch, {t:.1f} us per launch "
          f"-> {g / 8 / (t * 1e3):.2f} GHz")


if __name__ == "__main__":
    main()
