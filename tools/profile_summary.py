"""Turn tools/profile_round.sh output into the committed profiles/ files.

    python tools/profile_summary.py <round-tag>
writes profiles/<tag>_kernel_stats.csv (rocprofv3 --stats, mvn kernels; _cfgN: config N alone,
with that run's bench line as <tag>_bench_cfgN_traced.json), profiles/<tag>_traffic.json
(per config and kernel: mean FETCH_SIZE / WRITE_SIZE per dispatch; HBM bytes = 2 x FETCH + WRITE,
MI355X_MICROARCH.md 'HBM': gfx950 FETCH_SIZE counts half the bytes of wide streaming reads) and
profiles/<tag>_sq_cfg2.txt (SQ instruction mix of the unprojection).
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
raw = os.path.join(ROOT, "gpurun_out", tag)
dst = os.path.join(ROOT, "profiles")
os.makedirs(dst, exist_ok=True)


def short(name):
    name = name.replace("(anonymous namespace)::", "").replace("void ", "").replace("mvn::", "") \
        .replace("unproj::", "").replace("unsigned short", "bf16")
    return name.split("(")[0]


# 1. kernel stats: the whole bench, then one file per config (one config per traced process)
for sub, suffix in (("kt", ""), ("kt_cfg2", "_cfg2"), ("kt_cfg3", "_cfg3"), ("kt_cfg4", "_cfg4"),
                    ("kt_cfg2_fast", "_cfg2_fast"), ("kt_cfg3_fast", "_cfg3_fast")):
    stats = glob.glob(os.path.join(raw, sub, "**", "*kernel_stats.csv"), recursive=True)
    rows = [r for f in stats for r in csv.DictReader(open(f))]
    if not rows:
        continue
    with open(os.path.join(dst, f"{tag}_kernel_stats{suffix}.csv"), "w", newline="") as fo:
        w = csv.writer(fo)
        w.writerow(["kernel", "calls", "avg_us", "min_us", "max_us", "pct_of_gpu_time"])
        for r in rows:
            w.writerow([short(r["Name"]), r["Calls"], f"{float(r['AverageNs']) / 1e3:.2f}",
                        f"{float(r['MinNs']) / 1e3:.2f}", f"{float(r['MaxNs']) / 1e3:.2f}", r["Percentage"]])
    log = os.path.join(raw, sub + ".log")
    if suffix and os.path.exists(log):      # the traced run's own bench line
        lines = [ln for ln in open(log) if ln.startswith("{")]
        if lines:
            open(os.path.join(dst, f"{tag}_bench{suffix}_traced.json"), "w").write(lines[-1])

# 2. traffic
traffic = {}
for cfg in ("2", "3", "4"):
    per = defaultdict(dict)
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        vals = defaultdict(list)
        # pmc_<C>_cfgN (exact) and pmc_<C>_cfgN_fast (MVN_PRECISION_FAST): distinct kernel names
        for f in glob.glob(os.path.join(raw, f"pmc_{c}_cfg{cfg}*", "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                if r["Counter_Name"] == c:
                    vals[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
        for k, v in vals.items():
            per[k][c.lower() + "_kib"] = sum(v) / len(v)
            per[k]["dispatches"] = len(v)
    for k, d in per.items():
        if "fetch_size_kib" in d and "write_size_kib" in d:
            d["hbm_bytes_per_launch"] = (2 * d["fetch_size_kib"] + d["write_size_kib"]) * 1024
    traffic[f"cfg{cfg}"] = per
traffic["_note"] = ("rocprofv3 --pmc FETCH_SIZE and WRITE_SIZE in separate passes over tools/prof_unproject.py; "
                    "HBM bytes = 2 x FETCH_SIZE + WRITE_SIZE (KiB -> bytes), MI355X_MICROARCH.md 'HBM' gfx950 rule")
json.dump(traffic, open(os.path.join(dst, f"{tag}_traffic.json"), "w"), indent=1, sort_keys=True)

# 3. SQ mix (configs 2 and 3; config 3 also in the fast arithmetic), memory-pipe counters
for cfg in ("2", "3", "3_fast", "mem_cfg3", "mem_cfg3_fast", "mem_cfg4", "mem_cfg4_fast"):
    vals = defaultdict(lambda: defaultdict(list))
    sub = cfg if cfg.startswith("mem_") else f"sq_cfg{cfg}"
    for f in glob.glob(os.path.join(raw, sub, "p*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            vals[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    if not vals:
        continue
    with open(os.path.join(dst, f"{tag}_{sub}.txt"), "w") as fo:
        for k, d in vals.items():
            fo.write(k + "\n")
            waves = sum(d["SQ_WAVES"]) / len(d["SQ_WAVES"]) if "SQ_WAVES" in d else None
            for c in sorted(d):
                m = sum(d[c]) / len(d[c])
                per = f"   per wave {m / waves:12.1f}" if waves else ""
                fo.write(f"   {c:28s} {m:16.1f}{per}\n")
print(open(os.path.join(dst, f"{tag}_kernel_stats.csv")).read())
print(json.dumps(traffic, indent=1))

