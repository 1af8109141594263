"""Per-kernel totals of every counter in <dir>/p*/run_counter_collection.csv (development tool)."""
import csv
import glob
import os
import sys
from collections import defaultdict

tot = defaultdict(lambda: defaultdict(float))
calls = defaultdict(set)
for f in sorted(glob.glob(os.path.join(sys.argv[1], "p*", "run_counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("artes::", "")
        if "rocclr" in k:
            continue
        tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
        calls[k].add(r["Dispatch_Id"])
for k, c in tot.items():
    print(f"{k}  (dispatches {len(calls[k])})")
    for n, v in sorted(c.items()):
        print(f"   {n:28s} {v:.4e}")
