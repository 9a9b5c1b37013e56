"""Per-kernel duration summary from a rocprofv3 rocpd database (results.db), grouped by kernel
name and grid: python tools/rocpd_stats.py path/to/results.db [name-substring]"""
import sqlite3
import sys
from collections import defaultdict


def main():
    c = sqlite3.connect(sys.argv[1])
    sub = sys.argv[2] if len(sys.argv) > 2 else ""
    g = defaultdict(list)
    for name, gx, gy, gz, vg, d in c.execute(
            "select name, grid_x, grid_y, grid_z, vgpr_count, duration from kernels order by start"):
        if sub in name:
            g[(name[:90], gx, gy, gz, vg)].append(d / 1e3)
    print(f"{'kernel':90s} {'grid':>20s} {'vgpr':>5s} {'n':>5s} {'mean us':>9s} {'min us':>9s}")
    for (n, gx, gy, gz, vg), v in sorted(g.items(), key=lambda kv: -sum(kv[1])):
        print(f"{n:90s} {f'{gx}x{gy}x{gz}':>20s} {vg:5d} {len(v):5d} {sum(v) / len(v):9.1f} {min(v):9.1f}")


if __name__ == "__main__":
    main()
