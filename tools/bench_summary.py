"""Print the headline numbers of a bench.py JSON line (the file's first line that starts with "{")."""
import json
import sys

d = json.loads(next(l for l in open(sys.argv[1]) if l.startswith("{")))   # (gloo prints before the line)
rf = d.get("roofline", {})
print(f"value {d['value']} GB/s, {d['ms_per_step']} ms/step, n_gpus {d['n_gpus']}, self_check {d.get('self_check')}, "
      f"fast_path {d.get('decoder_fast_path')}")
print("kernels_ms", d.get("kernels_ms"))
print("roofline", {k: rf.get(k) for k in ("kernel", "achieved", "frac", "achievable", "frac_of_achievable", "traffic")})
if "end_to_end" in d:
    e = d["end_to_end"]
    print("end_to_end", e.get("value"), e.get("ms_per_step"), "self_check", e.get("self_check"))
for grp in ("sweep", "configs"):
    for k, v in d.get(grp, {}).items():
        print(grp, k, v.get("value"), v.get("ms_per_step"), "self_check", v.get("self_check"), "fast", v.get("fast_path"))
if "pipelined" in d:
    print("pipelined", d["pipelined"].get("value"), d["pipelined"].get("ms_per_step"))
if "cpu_baseline" in d:
    print("cpu_baseline", d["cpu_baseline"])
