"""Per-wave SQ counter summary of tools/pmc_sq.sh output.
    python tools/sq_summary.py <pmc_sq outdir>"""
import collections
import csv
import glob
import sys

vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{sys.argv[1]}/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        vals[r["Kernel_Name"].split("(")[0][-60:]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in vals.items():
    print(k)
    w = sum(d["SQ_WAVES"]) / len(d["SQ_WAVES"])
    for c in sorted(d):
        m = sum(d[c]) / len(d[c])
        print("  %-28s %16.1f  per wave %12.1f" % (c, m, m / w))
