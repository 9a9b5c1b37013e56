"""Sum each counter over the dispatches of a PMC output dir (rocprofv3 csv), per dispatch average.
    python tools/pmc_dump.py <outdir>"""
import csv
import glob
import os
import sys
from collections import defaultdict

tot, disp = defaultdict(float), defaultdict(set)
for f in glob.glob(os.path.join(sys.argv[1], "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        tot[r["Counter_Name"]] += float(r["Counter_Value"])
        disp[r["Counter_Name"]].add((f, r["Dispatch_Id"]))
for k in sorted(tot):
    print(f"{k:40s} {tot[k] / max(1, len(disp[k])):.4g}")
