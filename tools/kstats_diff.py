"""Per-kernel total time per step, two kernel-trace profiles of the same bench command
(tools/gpu_step_prof_ab.sh): the kernels whose time changed most. Usage: kstats_diff.py TAG [N]"""
import csv
import glob
import sys

tag = sys.argv[1]
top = int(sys.argv[2]) if len(sys.argv) > 2 else 15


def load(side):
    f = glob.glob(f"gpurun_out/{tag}_{side}/**/*kernel_stats.csv", recursive=True)[0]
    return {r["Name"][:90]: float(r["TotalDurationNs"]) / 1e3 for r in csv.DictReader(open(f))}


new, old = load("new"), load("old")
keys = set(new) | set(old)
rows = sorted(keys, key=lambda k: -abs(new.get(k, 0) - old.get(k, 0)))
print(f"{'kernel':90s} {'old us':>10s} {'new us':>10s} {'diff':>9s}")
for k in rows[:top]:
    print(f"{k:90s} {old.get(k, 0):10.1f} {new.get(k, 0):10.1f} {new.get(k, 0) - old.get(k, 0):9.1f}")
print(f"{'total':90s} {sum(old.values()):10.1f} {sum(new.values()):10.1f}")
