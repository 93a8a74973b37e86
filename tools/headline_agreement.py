"""Headline roofline agreement: the bench line's HIP-event time of the headline probe (MLP Dense_0
dW: split-K TN GEMM + combine, one mmt_gemm launch) against rocprofv3's kernel trace of the same
command (the probe launches after the last AdamW of the trace).
usage: headline_agreement.py TAG  (reads gpurun_out/TAG_benchprof/**/run_kernel_trace.csv and
profiles/TAG_bench.json; prints the profiles/TAG_headline_agreement.txt text)"""
import csv
import glob
import json
import statistics
import sys

tag = sys.argv[1]
tr = glob.glob(f"gpurun_out/{tag}_benchprof/**/run_kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(tr)), key=lambda r: int(r["Start_Timestamp"]))
last = max(i for i, r in enumerate(rows) if "adamw_kernel" in r["Kernel_Name"])
after = rows[last + 1:]


def durs(pat):
    return [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in after
            if pat in r["Kernel_Name"]]


line = json.load(open(f"profiles/{tag}_bench.json"))
roof = line["roofline"]
tn_name = "gemm_tn_dma16_kernel<384>"
tn = durs("gemm_tn_dma16_kernel<384>")
if not tn:
    tn_name, tn = "gemm_tn_r4_kernel<384>", durs("gemm_tn_r4_kernel<384>")
comb = durs("splitk_epilogue_kernel<1")
# the probe's launches: the TN kernels at the headline shape dominate after the last step; take
# the tail of the largest group (every probe launch repeats the same shape)
n = len(after)
tot = statistics.mean(tn) + statistics.mean(comb)
ev = roof["avg_launch_us"]
print(f"Headline roofline agreement ({tag}; source digest {roof['traffic_source'].split('digest ')[-1].rstrip(')')}):")
print(f"  {roof['kernel']}")
print(f"  rocprofv3 --kernel-trace --stats ({len(tn)} TN launches, {n} kernels after the last AdamW):")
print(f"    {tn_name} mean {statistics.mean(tn):.2f} us (median {statistics.median(tn):.2f}), "
      f"splitk_epilogue_kernel<1> mean {statistics.mean(comb):.2f} us")
print(f"    sum {tot:.1f} us")
print(f"  the bench line's HIP-event time over the same launch (un-profiled run, {tag}_bench.json):")
print(f"    {ev} us (the events also hold the gap between the two launches) -> frac {roof['frac']}")
print(f"  agreement: {abs(ev - tot) / ev * 100:.1f} %")
print(f"  traffic (PMC, {roof['traffic_source'].split(' (')[0]}): {roof['traffic'] / 1e6:.1f} MB per "
      f"launch against {roof['algorithmic_bytes_per_launch'] / 1e6:.1f} MB algorithmic")
print(f"step: {line['value']} samples/s, {line['ms_per_step']} ms/step")
