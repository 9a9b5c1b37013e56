"""Static instruction mix of kernels in a hipcc -save-temps assembly file.
    python tools/isa_mix.py file.s <mangled-name-substring> [<substring> ...]
Prints, per matching kernel, the count of each ds_* / buffer_* instruction, the SALU and
VALU totals and the most frequent SALU opcodes (static counts: loop bodies once)."""
import collections
import re
import sys


def kernels(path):
    text = open(path).read()
    for m in re.finditer(r"^(_Z\S+):\s*;\s*@", text, re.M):
        start = m.end()
        end = text.find(".Lfunc_end", start)
        yield m.group(1), text[start:end]


def main():
    path, subs = sys.argv[1], sys.argv[2:]
    for name, body in kernels(path):
        if subs and not any(s in name for s in subs):
            continue
        ops = collections.Counter(re.findall(r"^\s+([a-z_0-9]+)\s", body, re.M))
        print(name)
        print("  ds/buffer:", {k: v for k, v in sorted(ops.items()) if k.startswith(("ds_", "buffer_"))})
        print("  salu", sum(v for k, v in ops.items() if k.startswith("s_")),
              "valu", sum(v for k, v in ops.items() if k.startswith("v_")))
        print("  top salu:", sorted(((v, k) for k, v in ops.items() if k.startswith("s_")), reverse=True)[:16])


if __name__ == "__main__":
    main()
