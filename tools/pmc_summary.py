"""Summarise tools/pmc.sh output: per kernel, mean of each counter over dispatches."""
import csv
import glob
import os
import sys
from collections import defaultdict

root = sys.argv[1]
vals = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(root, "p*", "**", "*counter_collection.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        k = row["Kernel_Name"].split("(")[0][-60:]
        vals[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
for k, d in vals.items():
    print(k)
    for c in sorted(d):
        v = d[c]
        print(f"   {c:32s} {sum(v) / len(v):16.1f}   (n={len(v)})")
