"""Print the bench lines of one tools/cycle.sh run (local helper)."""
import json
import os
import sys

tag = sys.argv[1]
for name in ("bench", "book", "power"):
    f = f"gpurun_out/{tag}_{name}.json"
    if not os.path.exists(f):
        continue
    try:
        d = json.loads([l for l in open(f) if l.startswith("{")][0])
    except Exception as e:  # noqa
        print(name, "unreadable", e)
        continue
    print(name, f"{d['value']:.4g} spans/s", d["ms_per_step"], "ms/step  kern",
          d["roofline"]["kernel_ms_per_step"])
    print("   ", {k: v["ms_per_step"] for k, v in d["roofline"]["kernels"].items()})
f = f"gpurun_out/{tag}_diag.txt"
if os.path.exists(f):
    print("".join(l for l in open(f) if l.startswith("kmz")))
