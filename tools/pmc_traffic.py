#!/usr/bin/env python3
"""Turn two rocprofv3 --pmc passes over `bench.py --probe-only` into the per-launch HBM traffic
of every kernel probe (the `traffic` fields of bench.py's roofline).

    python bench.py --probe-only > gpurun_out/probes.json
    rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_fetch -o run --output-format csv -- python bench.py --probe-only
    rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc_write -o run --output-format csv -- python bench.py --probe-only
    python tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write --probes gpurun_out/probes.json --out profiles/r02_probe_pmc.json

FETCH_SIZE and WRITE_SIZE are in KB. gfx950 correction (MI355X_MICROARCH.md, "HBM"): FETCH_SIZE
counts half of the bytes of 16 B/lane streaming reads, so reads = 2 x FETCH_SIZE; WRITE_SIZE is
exact for 16 B/lane stores. A probe whose launch is several kernels (attention backward = dQ +
dK/dV, split-K GEMM + combine) is matched by its main kernel only.
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import re
import statistics


def per_dispatch(d: str, counter: str, kernel: str) -> list[float]:
    """Counter value per dispatch of the kernel, in dispatch order."""
    files = glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection csv under {d}")
    vals: dict[str, float] = {}
    # the probe's kernel name as a whole identifier ("seqnorm_fwd_kernel" must not match
    # "tome_merge_seqnorm_fwd_kernel"; a trailing "_" / "<" is a prefix match: "Cijk_")
    pat = re.compile(r"(?<![A-Za-z0-9_])" + re.escape(kernel))
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != counter or not pat.search(row.get("Kernel_Name", "")):
                    continue
                key = (f, int(row.get("Dispatch_Id") or 0))
                vals[key] = vals.get(key, 0.0) + float(row["Counter_Value"])
    return [vals[k] for k in sorted(vals)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("--probes", required=True, help="the JSON line of bench.py --probe-only")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    with open(a.probes) as fh:
        line = [ln for ln in fh if ln.startswith("{")][-1]
    meta = json.loads(line)
    probes = meta["probes"]
    res = {}
    # probes that share a kernel (the two residual-stream products on gemm_glds_nt_kernel) ran
    # one after the other: the k-th of them owns the k-th contiguous share of the dispatches
    share = {}
    for p in probes:
        share.setdefault(p["kernel"], []).append(p["name"])

    def part(vals, p):
        names = share[p["kernel"]]
        n, k = len(names), names.index(p["name"])
        if n == 1:
            return vals
        m = len(vals) // n
        return vals[k * m:(k + 1) * m]
    for p in probes:
        fetch = part(per_dispatch(a.fetch_dir, "FETCH_SIZE", p["kernel"]), p)
        write = part(per_dispatch(a.write_dir, "WRITE_SIZE", p["kernel"]), p)
        if not fetch or not write:
            print(f"no counter rows for {p['kernel']}")
            continue
        f_kb, w_kb = statistics.median(fetch), statistics.median(write)
        hbm = 2 * f_kb * 1024 + w_kb * 1024
        alg = p.get("bytes_per_launch") or p.get("algorithmic_bytes_per_launch")
        res[p["name"]] = dict(kernel=p["kernel"], dispatches=[len(fetch), len(write)],
                              fetch_size_kb_median=f_kb, write_size_kb_median=w_kb,
                              read_bytes_corrected=2 * f_kb * 1024, write_bytes=w_kb * 1024,
                              hbm_bytes_per_launch=round(hbm), algorithmic_bytes_per_launch=alg,
                              ratio_to_algorithmic=round(hbm / alg, 3) if alg else None)
    with open(a.out, "w") as fh:
        json.dump(dict(batch=meta.get("batch", 256), source_digest=meta.get("source_digest"),
                       probes=res), fh, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
