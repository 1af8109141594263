"""Sum rocprofv3 --pmc counters per artes kernel: python tools/pmc_kernels.py <run_counter_collection.csv>"""
import csv
import sys
from collections import defaultdict

t = defaultdict(lambda: defaultdict(float))
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("artes::", "")
    t[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, c in t.items():
    if k.startswith("k_"):
        print(f"{k}: " + " ".join(f"{n}={v:.4g}" for n, v in sorted(c.items())))
