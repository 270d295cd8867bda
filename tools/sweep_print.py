"""Print the retrieval legs' call-level figures and Q sweeps from a bench.py log."""
import json
import sys

line = [x for x in open(sys.argv[1]) if x.startswith("{")][0]
d = json.loads(line)
for key, v in d.items():
    if not (isinstance(v, dict) and "call_level" in v):
        continue
    cl = v["call_level"]
    print(f"{key}: serial call {cl['serial_us_per_call']:.1f} us = {cl['serial_hbm_frac']:.3f}, "
          f"filter {cl['filter_hbm_frac']:.3f}")
    for q in v.get("q_sweep_local") or []:
        print(f"   Q={q['Q']:4d} filter {q['filter_us']:7.1f} us ({q['hbm_frac']:.3f})  "
              f"call {q['call_us']:7.1f} us ({q['call_hbm_frac']:.3f})")
