"""One C3 query's dispatches, in order, from a rocprofv3 kernel trace (per-launch durations and grid
sizes, which the per-kernel stats average away):   python3 tools/trace_launches.py TRACEDIR [MIN_US]
The query is the trace's last one: it starts at the last filter scan (uscan_kernel)."""
import csv
import glob
import os
import re
import sys

d = sys.argv[1]
min_us = float(sys.argv[2]) if len(sys.argv) > 2 else 5.0
rows = []
for fn in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
    rows += list(csv.DictReader(open(fn)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if "uscan_kernel" in r["Kernel_Name"]]
q = rows[starts[-1]:] if starts else rows
gkey = next((k for k in (q[0].keys() if q else []) if k.lower().startswith("grid_size")), None)
wkey = next((k for k in (q[0].keys() if q else []) if k.lower().startswith("workgroup_size")), None)
t0 = int(q[0]["Start_Timestamp"]) if q else 0
tot = 0.0
for r in q:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    us = (e - s) / 1e3
    tot += us
    if us < min_us:
        continue
    name = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "")[:100]
    print(f"{(s - t0) / 1e3:9.1f} {us:8.1f} us  grid {r.get(gkey, '?'):>9} wg {r.get(wkey, '?'):>5}  {name}")
print(f"query: {len(q)} dispatches, kernel time {tot / 1e3:.3f} ms, span {(int(q[-1]['End_Timestamp']) - t0) / 1e6:.3f} ms"
      if q else "no dispatches")
