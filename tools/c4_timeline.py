"""Summarise a rocprofv3 kernel trace over the window tools/c4_once.py stamped: GPU busy fraction,
mean concurrency, dispatch count and per-kernel time.   python3 tools/c4_timeline.py TRACEDIR STAMPFILE"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict

d, stamp = sys.argv[1], sys.argv[2]
t0, t1 = map(int, open(stamp).read().split())
files = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
ev = []
for fn in files:
    for r in csv.DictReader(open(fn)):
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if s >= t0 and e <= t1:
            ev.append((s, e, re.sub(r"\(.*", "", r["Kernel_Name"])[:90]))
ev.sort()
span = t1 - t0
busy, cur_s, cur_e = 0, None, None
for s, e, _ in ev:
    if cur_e is None or s > cur_e:
        if cur_e is not None:
            busy += cur_e - cur_s
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
if cur_e is not None:
    busy += cur_e - cur_s
tot = sum(e - s for s, e, _ in ev)
print(f"window {span / 1e6:.1f} ms, {len(ev)} dispatches, GPU busy (any kernel) {busy / span:.3f}, "
      f"mean concurrency while busy {tot / max(busy, 1):.2f}, kernel-time sum {tot / 1e6:.1f} ms")
durs = sorted(e - s for s, e, _ in ev)
for q in (0.1, 0.5, 0.9, 0.99):
    print(f"  dispatch duration p{int(q * 100)}: {durs[int(q * (len(durs) - 1))] / 1e3:.1f} us")
per = defaultdict(lambda: [0, 0])
for s, e, n in ev:
    per[n][0] += e - s
    per[n][1] += 1
for n, (t, c) in sorted(per.items(), key=lambda kv: -kv[1][0])[:25]:
    print(f"  {t / 1e6:8.2f} ms {c:7d} x {t / c / 1e3:7.1f} us  {n}")
