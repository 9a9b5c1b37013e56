"""Where a bench step's time goes between its kernels: from a rocprofv3 --kernel-trace CSV of
bench.py, the steps (unprojection -> soft-argmax partials -> combine -> finalize, back to back
on one stream) are found and the medians of each kernel's duration, each gap between
consecutive kernels of a step, the gap to the next step's first kernel, and the step period
are printed (ns).   python tools/step_gaps.py kt_kernel_trace.csv [unproject-name-substring]"""
import csv
import statistics
import sys

KINDS = ("unproject_", "softargmax_partials", "softargmax_combine", "softargmax_finalize")


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    want = sys.argv[2] if len(sys.argv) > 2 else "unproject_x4"
    kind = [next((k for k in KINDS if k in r["Kernel_Name"]), None) for r in rows]
    steps = []
    for i in range(len(rows) - 4):
        if want in rows[i]["Kernel_Name"] and kind[i:i + 4] == list(KINDS):
            s = [int(rows[i + k]["Start_Timestamp"]) for k in range(5)]
            e = [int(rows[i + k]["End_Timestamp"]) for k in range(4)]
            steps.append((s, e, kind[i + 4] == KINDS[0]))
    med = statistics.median
    print(f"steps found: {len(steps)}")
    for k in range(4):
        print(f"  {KINDS[k]:22s} duration {med(e[k] - s[k] for s, e, _ in steps):9.0f} ns")
    for k in range(3):
        print(f"  gap {KINDS[k]:>20s} -> next {med(s[k + 1] - e[k] for s, e, _ in steps):7.0f} ns")
    nxt = [s[4] - e[3] for s, e, ok in steps if ok]
    if nxt:
        print(f"  gap finalize -> next step's unprojection {med(nxt):7.0f} ns")
        print(f"  step period (unprojection start to start) {med(s[4] - s[0] for s, e, ok in steps if ok):9.0f} ns")
        print(f"  kernel sum {med(sum(e[k] - s[k] for k in range(4)) for s, e, ok in steps if ok):9.0f} ns")


if __name__ == "__main__":
    main()
