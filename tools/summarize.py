"""Print the summary of one tools/gpu_cycle.sh run (local helper)."""
import csv
import json
import sys

tag = sys.argv[1]
print(open(f"gpurun_out/t_{tag}.log").read().strip().splitlines()[-2:])
for name in ("mesh", "book"):
    try:
        line = [l for l in open(f"gpurun_out/bench_{name}_{tag}.json") if l.startswith("{")][0]
        d = json.loads(line)
        print(name, f"{d['value']:.3e} spans/s", d["ms_per_step"], "ms/step", d["roofline"]["kernel"], d["roofline"]["frac"],
              {k: v["avg_ms"] for k, v in d["roofline"]["kernels"].items()})
    except Exception as e:  # noqa
        print(name, "missing", e)
try:
    for x in list(csv.DictReader(open(f"gpurun_out/prof_{tag}/mesh_kernel_stats.csv")))[:12]:
        print(x["Name"][:50].ljust(52), x["Calls"].rjust(4), "%10.1f us" % (float(x["AverageNs"]) / 1e3))
except Exception as e:  # noqa
    print("no profile", e)
