"""Print the key numbers of the last tools/gpu_check.sh run (gpurun_out/)."""
import json
import os
import subprocess
import sys

OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out")


def tail(name, n=2):
    p = os.path.join(OUT, name)
    if os.path.exists(p):
        print(f"--- {name}:", *open(p).read().splitlines()[-n:], sep="\n")


tail("pytest_gpu.log")
p = os.path.join(OUT, "gemm_bench.log")
if os.path.exists(p):
    print("--- gemm_bench:")
    print("\n".join(l for l in open(p).read().splitlines() if "amdgpu.ids" not in l))
p = os.path.join(OUT, "bench.log")
if os.path.exists(p):
    lines = [l for l in open(p).read().splitlines() if l.startswith("{")]
    if lines:
        d = json.loads(lines[-1])
        print("--- bench: value", round(d["value"], 1), d["unit"], "ms/step", round(d["ms_per_step"], 3),
              "roofline", d["roofline"].get("achieved"), d["roofline"].get("frac"))
        if "train" in d:
            print("    train step TF/s", round(d["train"]["step_tflops"], 1))
        r = d.get("retrieval")
        if r:
            print("    scan q/s", round(r["value"]), "filter GB/s", r["roofline"]["achieved"],
                  "us", r["roofline"]["kernel_avg_us"])
            for x in r.get("q_sweep_local") or []:
                print("     ", {k: (round(v, 3) if isinstance(v, float) else v) for k, v in x.items()})
    else:
        tail("bench.log", 15)
if len(sys.argv) > 1:
    subprocess.run([sys.executable, os.path.join(os.path.dirname(__file__), "prof_summary.py"),
                    os.path.join(OUT, sys.argv[1])])
