#!/usr/bin/env python3
"""Instruction mix per kernel of a hipcc -S (device-only) assembly file.
Usage: isa_mix.py FILE.s [NAME_SUBSTR ...]"""
import collections
import re
import sys


def kernels(path):
    s = open(path).read()
    for m in re.finditer(r"^(_Z\S+):[^\n]*\n(.*?)^\.Lfunc_end", s, re.M | re.S):
        yield m.group(1), m.group(2)


def main():
    path, subs = sys.argv[1], sys.argv[2:]
    for name, body in kernels(path):
        if subs and not any(x in name for x in subs):
            continue
        ins = re.findall(r"^\s+([sv]_[a-z0-9_]+|ds_[a-z0-9_]+|global_[a-z0-9_]+|buffer_[a-z0-9_]+|scratch_[a-z0-9_]+)", body, re.M)
        c = collections.Counter(ins)
        mf = sum(v for k, v in c.items() if "mfma" in k)
        valu = sum(v for k, v in c.items() if k.startswith("v_") and "mfma" not in k)
        top = ", ".join(f"{k} {v}" for k, v in c.most_common(40) if k.startswith("v_") and "mfma" not in k)
        vg = re.search(r"\.vgpr_count:\s+(\d+)", body)
        print(f"{name[:90]}\n  static: mfma {mf} valu {valu} ds {sum(v for k, v in c.items() if k.startswith('ds_'))}"
              f" scratch {sum(v for k, v in c.items() if k.startswith('scratch_'))}\n  {top}")


if __name__ == "__main__":
    main()
