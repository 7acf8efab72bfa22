"""Summarise an ab_variants.sh run: ms/step and per-kernel ms per variant."""
import glob, json, os, sys
d = sys.argv[1]
keys = sys.argv[2].split(",") if len(sys.argv) > 2 else ["walk", "join", "cert", "check", "stats", "reduce", "settle"]
for f in sorted(glob.glob(os.path.join(d, "*.json"))):
    try:
        j = json.loads([l for l in open(f) if l.startswith("{")][-1])
    except Exception as e:
        print(os.path.basename(f), "no line", e); continue
    k = j["roofline"]["kernels"]
    print("%-22s %.4f " % (os.path.basename(f), j["ms_per_step"]) + " ".join("%s=%.3f" % (x, k[x]["avg_ms"]) for x in keys if x in k), "frac=%.3f" % j["roofline"]["frac"])
