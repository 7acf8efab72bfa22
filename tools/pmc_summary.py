"""Summarise rocprofv3 --pmc counter CSVs: mean counter value per kernel."""
import csv
import sys
from collections import defaultdict

acc = defaultdict(lambda: defaultdict(list))
for path in sys.argv[1:]:
    with open(path) as f:
        for r in csv.DictReader(f):
            name = r["Kernel_Name"].split("(")[0][:48]
            acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
            acc[name]["_ns"].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
for k, d in sorted(acc.items()):
    if "copyBuffer" in k or "fill" in k.lower() and "synth" not in k:
        continue
    row = {c: sum(v) / len(v) for c, v in d.items()}
    print(k, {c: (f"{x:.4g}") for c, x in sorted(row.items())})
