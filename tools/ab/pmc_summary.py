"""Summarise a rocprofv3 --pmc sqlite result: per kernel, counter sums per dispatch (averaged)."""
import collections
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for name, ctr, disp, val in c.execute("select kernel_name, counter_name, dispatch_id, value from counters_collection"):
    acc[name.split("(")[0]][ctr].append((disp, val))
for k, d in acc.items():
    print(k)
    for ctr, v in sorted(d.items()):
        per = collections.defaultdict(float)
        for disp, x in v:
            per[disp] += x
        vals = list(per.values())
        print(f"  {ctr:28s} {sum(vals) / len(vals):16.4g}  (dispatches {len(vals)})")
