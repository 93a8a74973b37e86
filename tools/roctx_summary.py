#!/usr/bin/env python3
"""Per-phase summary of a `rocprofv3 --marker-trace --kernel-trace` run of an eager step
(MMT_ROCTX=1 python bench.py --no-graph ...): for every roctx range name (multi_modal_transformers_
tokenmerge_amd/tracing.py phases), the host-side range duration and the GPU time of the kernels
that started inside it (by kernel start timestamp), median over the occurrences.

    python tools/roctx_summary.py DIR [--out FILE]"""
import argparse
import collections
import csv
import glob
import os
import statistics


def rows(d, pat):
    out = []
    for f in glob.glob(os.path.join(d, "**", pat), recursive=True):
        with open(f) as fh:
            out += list(csv.DictReader(fh))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--out")
    a = ap.parse_args()
    marks = rows(a.dir, "*marker_api_trace.csv")
    kerns = rows(a.dir, "*kernel_trace.csv")
    ks = sorted((int(k["Start_Timestamp"]), int(k["End_Timestamp"])) for k in kerns)
    ranges = collections.defaultdict(list)
    for m in marks:
        name = m.get("Function") or m.get("Operation") or ""
        if m.get("Kind", "").upper().endswith("MARKER") or "Start_Timestamp" in m:
            try:
                s, e = int(m["Start_Timestamp"]), int(m["End_Timestamp"])
            except (KeyError, ValueError):
                continue
            if e > s and name:
                gpu = sum(ke - kb for kb, ke in ks if s <= kb < e)
                nk = sum(1 for kb, _ in ks if s <= kb < e)
                ranges[name].append((e - s, gpu, nk))
    lines = [f"{'phase':34s} {'n':>3s} {'host ms':>9s} {'kernel ms':>10s} {'kernels':>8s}"]
    for name, v in sorted(ranges.items(), key=lambda kv: -statistics.median(x[1] for x in kv[1])):
        lines.append(f"{name:34s} {len(v):3d} {statistics.median(x[0] for x in v) / 1e6:9.3f} "
                     f"{statistics.median(x[1] for x in v) / 1e6:10.3f} {int(statistics.median(x[2] for x in v)):8d}")
    txt = "\n".join(lines)
    print(txt)
    if a.out:
        with open(a.out, "w") as fh:
            fh.write(txt + "\n")


if __name__ == "__main__":
    main()
