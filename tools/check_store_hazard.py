"""Scan gfx950 assembly for a VMEM store of more than 8 bytes (dwordx3 / dwordx4) whose
data VGPRs a vector ALU instruction overwrites within the next WAIT_STATES (2) wait states.
Such a store can read the NEW value (observed: channels-last unprojection, r14, channels 14-15
nondeterministic), so every hit is a bug to fix in the source (a wait state / s_nop).
Wait states after the store: every issued instruction counts one, `s_nop N` counts N + 1;
an instruction is in the hazard window while fewer than WAIT_STATES have passed before it.
    python tools/check_store_hazard.py file.s|file.dis|lib.so [...]
A shared library is unbundled (llvm-objdump --offloading, in a temporary directory) and its
gfx950 code objects disassembled first; __graft_entry__.build() runs this on libmvn_hip.so."""
import glob
import os
import re
import shutil
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
WAIT_STATES = 2          # gfx940-class: a VALU write within 2 wait states of the store is a hazard

STORE = re.compile(r"^\s*(buffer|global|flat)_store_dwordx([34])\s+(v\[(\d+):(\d+)\]|v(\d+)),?\s*(v\[(\d+):(\d+)\]|v\d+)?")
DEST = re.compile(r"^\s*(v_[a-z0-9_]+)\s+v(?:\[(\d+):(\d+)\]|(\d+))")
NOP = re.compile(r"^\s*s_nop\s+(0x[0-9a-fA-F]+|\d+)")


def data_regs(m):
    # buffer_store_dwordxN vdata, vaddr, ... ; global_store_dwordxN vaddr, vdata, off
    kind = m.group(1)
    if kind == "buffer":
        lo, hi = int(m.group(4)), int(m.group(5))
    else:
        if m.group(8) is None:
            return set()
        lo, hi = int(m.group(8)), int(m.group(9))
    return set(range(lo, hi + 1))


def disassemble(so_path, tmp):
    """The gfx950 code objects of a HIP shared library, disassembled, as text files."""
    local = os.path.join(tmp, os.path.basename(so_path))
    shutil.copy(so_path, local)
    subprocess.run([f"{LLVM}/llvm-objdump", "--offloading", local], cwd=tmp, check=True, capture_output=True)
    out = []
    for co in sorted(glob.glob(local + ".*gfx950*")):
        dis = co + ".dis"
        with open(dis, "w") as f:
            subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--mcpu=gfx950", co], stdout=f, check=True)
        out.append(dis)
    return out


def scan(paths):
    hits = 0
    for path in paths:
        lines = open(path).read().splitlines()
        fn = "?"
        for i, ln in enumerate(lines):
            if re.match(r"^_Z\S*:", ln):
                fn = ln.split(":")[0]
            m = STORE.match(ln)
            if not m:
                continue
            regs = data_regs(m)
            waited, j = 0, i + 1
            while j < len(lines) and waited < WAIT_STATES:
                ln2 = lines[j].strip()
                j += 1
                if not ln2 or ln2.startswith(";") or ln2.endswith(":"):
                    continue                        # blank, comment, label
                nop = NOP.match(ln2)
                if nop:
                    waited += int(nop.group(1), 0) + 1
                    continue
                d = DEST.match(ln2)
                if d:
                    w = {int(d.group(4))} if d.group(4) is not None else set(range(int(d.group(2)), int(d.group(3)) + 1))
                    if w & regs:
                        hits += 1
                        print(f"{path}:{i + 1}: {fn[:90]}\n    {ln.strip()}\n    {ln2} (after {waited} wait state(s))")
                        break
                waited += 1
    return hits


def check(paths):
    """Number of hazards in the given .s / .dis files and shared libraries."""
    with tempfile.TemporaryDirectory() as tmp:
        files = []
        for p in paths:
            files += disassemble(p, tmp) if p.endswith(".so") else [p]
        return scan(files)


def main():
    hits = check(sys.argv[1:])
    print(f"{hits} hazard(s)")
    return 1 if hits else 0


if __name__ == "__main__":
    sys.exit(main())
