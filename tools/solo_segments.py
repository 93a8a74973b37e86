"""Where in a step one queue runs alone: over the last step of a rocprofv3 kernel trace (step
boundary = the AdamW launch), the maximal intervals during which exactly one hardware queue has a
kernel running, with their offset from the step start, their queue and the kernels they hold.
usage: solo_segments.py run_kernel_trace.csv [min_us]"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
min_us = float(sys.argv[2]) if len(sys.argv) > 2 else 20.0
ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r["Queue_Id"]), r["Kernel_Name"])
             for r in rows), key=lambda x: x[0])
ad = [k for k in ks if "adamw_kernel" in k[3]]
t0, t1 = ad[-2][1], ad[-1][1]
win = [k for k in ks if k[0] >= t0 and k[1] <= t1]
ev = []
for s, e, q, n in win:
    ev += [(s, 1, q), (e, -1, q)]
ev.sort(key=lambda x: (x[0], x[1]))
active = defaultdict(int)
segs = []          # (start, end, queue) of single-queue intervals
cur = None
last = t0
for t, d, q in ev:
    live = [k for k, v in active.items() if v > 0]
    if len(live) == 1:
        if cur and cur[2] == live[0] and cur[1] == last:
            cur[1] = t
        else:
            if cur:
                segs.append(tuple(cur))
            cur = [last, t, live[0]]
    last = t
    active[q] += d
if cur:
    segs.append(tuple(cur))
span = (t1 - t0) / 1e3
per_q = defaultdict(float)
for s, e, q in segs:
    per_q[q] += (e - s) / 1e3
print(f"step span {span:.1f} us; single-queue time by queue (us): "
      + ", ".join(f"q{q} {v:.0f}" for q, v in sorted(per_q.items())))
# main queue = the one that runs AdamW
mq = ad[-1][2]
print(f"main queue q{mq}")
for s, e, q in segs:
    if (e - s) / 1e3 < min_us:
        continue
    names = defaultdict(float)
    for ks_, ke, kq, n in win:
        if kq == q and ke > s and ks_ < e:
            names[n.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][:60]] += (min(ke, e) - max(ks_, s)) / 1e3
    top = sorted(names.items(), key=lambda x: -x[1])[:3]
    print(f"  +{(s - t0) / 1e3:8.1f} us  {(e - s) / 1e3:7.1f} us  q{q}  "
          + "; ".join(f"{n} {v:.0f}" for n, v in top))
