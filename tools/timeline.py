"""Per-step timeline of a rocprofv3 kernel trace (bench.py --no-probes): busy time per queue, the
union of all queues (GPU busy) and the idle gaps, over the last complete steps. The step boundary
is the AdamW launch. Usage: timeline.py run_kernel_trace.csv [steps]"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
nsteps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r["Queue_Id"]), r["Kernel_Name"])
             for r in rows), key=lambda x: x[0])
ad = [k for k in ks if "adamw_kernel" in k[3]]
t0, t1 = ad[-1 - nsteps][1], ad[-1][1]
win = [k for k in ks if k[0] >= t0 and k[1] <= t1]
per_q = defaultdict(int)
for s, e, q, n in win:
    per_q[q] += e - s
iv = sorted((s, e) for s, e, q, n in win)
busy, cur_s, cur_e, gaps = 0, iv[0][0], iv[0][1], []
for s, e in iv[1:]:
    if s > cur_e:
        busy += cur_e - cur_s
        gaps.append((s - cur_e, cur_e))
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += cur_e - cur_s
span = t1 - t0
print(f"{nsteps} steps: span {span / nsteps / 1e6:.3f} ms/step, GPU busy (any queue) {busy / nsteps / 1e6:.3f}, "
      f"idle {(span - busy) / nsteps / 1e6:.3f}")
for q, v in sorted(per_q.items()):
    print(f"  queue {q}: {v / nsteps / 1e6:.3f} ms/step of kernel time")
gaps.sort(reverse=True)
print("largest idle gaps (us):", [round(g / 1e3, 1) for g, _ in gaps[:10]])
# serial-only time: intervals where exactly one kernel runs, by kernel
ev = []
for s, e, q, n in win:
    ev += [(s, 1, n), (e, -1, n)]
ev.sort(key=lambda x: (x[0], x[1]))
active = defaultdict(int)
solo = defaultdict(int)
last = ev[0][0]
for t, d, n in ev:
    live = [k for k, v in active.items() if v > 0]
    if len(live) == 1:
        solo[live[0]] += t - last
    last = t
    active[n] += d
print("kernel time with nothing else running (ms/step):")
for n, v in sorted(solo.items(), key=lambda x: -x[1])[:25]:
    print(f"  {v / nsteps / 1e3:8.1f} us  {n[:110]}")
if "--gaps" in sys.argv:
    # kernels around each gap > 5 us (by end time before / start time after)
    ends = sorted(win, key=lambda k: k[1])
    for g, at in sorted(gaps, key=lambda x: x[1]):
        if g < 5000:
            continue
        before = max((k for k in win if k[1] <= at), key=lambda k: k[1])
        after = min((k for k in win if k[0] >= at + g), key=lambda k: k[0])
        print(f"gap {g / 1e3:6.1f} us  q{before[2]} {before[3][:60]:60s} -> q{after[2]} {after[3][:60]}")
