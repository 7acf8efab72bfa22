"""Print one bench step's GPU timeline (kernels + copies) with the gaps
between them, from a rocprofv3 --kernel-trace --memory-copy-trace csv run."""
import csv
import sys

d = sys.argv[1]
ev = []
for r in csv.DictReader(open(f"{d}/tl_kernel_trace.csv")):
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K:" + r["Kernel_Name"].split("(")[0][-30:]))
try:
    for r in csv.DictReader(open(f"{d}/tl_memory_copy_trace.csv")):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "C:" + r["Direction"] + ":" + r.get("Size", "?")))
except FileNotFoundError:
    pass
ev.sort()
starts = [i for i, e in enumerate(ev) if "k3_produce" in e[2]]
a, b = starts[-2], starts[-1]
prev, t0, busy = None, ev[a][0], 0
for e in ev[a:b + 1]:
    gap = (e[0] - prev) / 1000 if prev else 0
    print(f"{(e[0] - t0) / 1000:9.1f} +gap {gap:7.1f}  dur {(e[1] - e[0]) / 1000:8.1f}  {e[2]}")
    busy += e[1] - e[0]
    prev = e[1]
print(f"step {(ev[b][0] - t0) / 1000:.1f} us, busy {(busy - (ev[b][1] - ev[b][0])) / 1000:.1f} us")
