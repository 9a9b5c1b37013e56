"""Print VGPR / SGPR / scratch / occupancy per kernel of one .hip file (hipcc remarks)."""
import re
import subprocess
import sys

src = sys.argv[1]
extra = sys.argv[2:]
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fno-slp-vectorize",
       "-I/root/repo/include", "-I/root/repo/learnable-triangulation-pytorch_amd/csrc", "-c", src, "-o", "/tmp/_kr.o",
       "-Rpass-analysis=kernel-resource-usage"] + extra
out = subprocess.run(cmd, capture_output=True, text=True).stderr
cur = {}
rows = []
for line in out.splitlines():
    m = re.search(r"remark:\s+(Function Name|VGPRs|TotalSGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (\S+)", line)
    if not m:
        continue
    k, v = m.groups()
    if k == "Function Name":
        if cur:
            rows.append(cur)
        cur = {"name": v}
    else:
        cur[k.split()[0]] = v
if cur:
    rows.append(cur)
dem = subprocess.run(["c++filt"], input="\n".join(r["name"] for r in rows), capture_output=True, text=True).stdout.split("\n")
for r, d in zip(rows, dem):
    d = d.replace("(anonymous namespace)::", "").replace("mvn::", "").replace("unsigned short", "bf16")
    d = re.sub(r"\(.*", "", d)
    print(f"{d:70s} vgpr={r.get('VGPRs'):>4} sgpr={r.get('TotalSGPRs'):>4} scratch={r.get('ScratchSize'):>3} occ={r.get('Occupancy')} lds={r.get('LDS')}")
