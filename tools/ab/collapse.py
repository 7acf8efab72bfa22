"""Collapse A/B evidence: every bench line (*.json) under a directory into
one SUMMARY.json (per file: ms/step, per-kernel avg ms, roofline frac and the
config), then remove the raw lines.  Keeps the numbers DESIGN.md cites while
the directory stops holding one file per run.  usage: collapse.py DIR [DIR..]"""
import glob
import json
import os
import sys


def line(path):
    try:
        txt = open(path).read()
    except OSError:
        return None
    for l in reversed(txt.splitlines()):
        if l.startswith("{"):
            try:
                return json.loads(l)
            except ValueError:
                pass
    try:
        return json.loads(txt)
    except ValueError:
        return None


for d in sys.argv[1:]:
    out, gone = {}, []
    for f in sorted(glob.glob(os.path.join(d, "**", "*.json"), recursive=True)):
        if os.path.basename(f) == "SUMMARY.json":
            continue
        j = line(f)
        rel = os.path.relpath(f, d)
        if not isinstance(j, dict) or "ms_per_step" not in j:
            out[rel] = j  # (not a bench line: kept whole)
        else:
            r = j.get("roofline", {})
            out[rel] = {"ms_per_step": j["ms_per_step"], "value": j.get("value"),
                        "workload": j.get("config", {}).get("workload"),
                        "frac": r.get("frac"), "kernel": r.get("kernel"),
                        "kernels_avg_ms": {k: v.get("avg_ms") for k, v in r.get("kernels", {}).items()}}
        gone.append(f)
    if not out:
        continue
    prev = os.path.join(d, "SUMMARY.json")
    if os.path.exists(prev):
        out = {**json.load(open(prev)), **out}
    json.dump(out, open(prev, "w"), indent=1, sort_keys=True)
    for f in gone:
        os.remove(f)
    print(d, len(gone), "files ->", prev)
