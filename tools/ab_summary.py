"""Summary of tools/gpu_step_ab.sh logs: step value and probe launch times per build and round.
Usage: ab_summary.py TAG"""
import glob
import json
import sys

tag = sys.argv[1]
for f in sorted(glob.glob(f"gpurun_out/{tag}_*[0-9].log")):
    for line in open(f):
        if line.startswith("{"):
            d = json.loads(line)
            ks = d.get("roofline", {}).get("kernels", [])
            print(f"{f.split('/')[-1]:28s} {d['value']:9.1f}  " +
                  " ".join(f"{k['name']}={k['avg_launch_us']:.1f}" for k in ks))
for f in sorted(glob.glob(f"gpurun_out/{tag}_t5*.log")):
    print(f, [l.strip() for l in open(f) if "T5" in l])
