"""One-screen summary of a bench.py JSON line: headline, roofline, each config, parity."""
import json
import sys


def main():
    d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
    r = d.get("roofline") or {}
    print(f"headline {d['value']:.0f} {d['unit']} ({d.get('precision')}), {d['ms_per_step'] * 1e3:.1f} us/step; "
          f"unproject {(r.get('launch_ms') or 0) * 1e3:.1f} us frac {r.get('frac')}, softargmax {d.get('softargmax_ms')}")
    print("  parity", d.get("parity"))
    s = d.get("secondary") or {}
    if s:
        print(f"cfg3 {s['value']:.0f} unproject {s['unproject_ms'] * 1e3:.1f} us frac {s['roofline']['frac']:.3f} "
              f"sa {s['softargmax_ms'] * 1e3:.1f}  parity {s.get('parity', {}).get('unproject_max_rel')}")
    o = d.get("other_precision") or {}
    for k in ("config2", "config3"):
        if k in o:
            x = o[k]
            print(f"{o['precision']} {k} {x['value']:.0f} unproject {x['unproject_ms'] * 1e3:.1f} us frac "
                  f"{x['roofline']['frac']:.3f} sa {x['softargmax_ms'] * 1e3:.1f}  parity "
                  f"{ {kk: vv for kk, vv in (x.get('parity') or {}).items() if 'rel' in kk or 'bar' in kk} }")
    for k in ("config4", "config5", "config1", "in_kernel_coords"):
        x = d.get(k) or {}
        if x:
            print(k, {kk: x[kk] for kk in ("value", "ms_per_step", "unproject_ms", "unproject_frac") if kk in x},
                  (x.get("roofline") or {}).get("frac"))
    print("cpu_baseline", (d.get("cpu_baseline") or {}).get("value"), "dist", d.get("dist", {}).get("distinct_devices"))


if __name__ == "__main__":
    main()
