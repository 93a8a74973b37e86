#!/usr/bin/env python3
"""Register / spill metadata per kernel from a hipcc -S assembly file. Usage: kmeta.py FILE.s [SUBSTR]"""
import re
import sys

s = open(sys.argv[1]).read()
sub = sys.argv[2] if len(sys.argv) > 2 else ""
for blk in re.split(r"\n\s+- \.agpr_count", s)[1:]:
    name = re.search(r"\.name:\s+(\S+)", blk)
    if not name or sub not in name.group(1):
        continue
    f = {k: re.search(rf"\.{k}:\s+(\d+)", blk) for k in ("sgpr_count", "sgpr_spill_count", "vgpr_count", "vgpr_spill_count")}
    print(f"{name.group(1)[15:95]:80s} " + " ".join(f"{k}={v.group(1) if v else '?'}" for k, v in f.items()))
