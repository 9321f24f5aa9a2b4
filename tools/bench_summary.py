"""Print the headline and secondary numbers of a bench.py JSON line (argv[1])."""
import json
import sys

d = json.load(open(sys.argv[1]))
sec = d.pop("secondary", None) or {}
print("value", d["value"], "ms/step", d["ms_per_step"], "kernel_ms", d["kernel_ms"], "frac", d["roofline"]["frac"])
for k, v in sec.items():
    print(k, {kk: vv for kk, vv in v.items() if kk not in ("workload", "path", "cpu_baseline")}, v.get("cpu_baseline"))
