#!/usr/bin/env python3
"""print the key fields of bench JSON lines in log files (tuning aid)"""
import json
import sys

for fn in sys.argv[1:]:
    try:
        line = [l for l in open(fn).read().splitlines() if l.startswith("{")][-1]
        d = json.loads(line)
    except Exception as e:  # noqa: BLE001
        print(f"{fn}: no line ({e.__class__.__name__})")
        continue
    print(f"{fn}: value {d['value']} ms/step {d['ms_per_step']} parity {d.get('parity')}")
    for k in ("other_executors_same_batch", "stages", "stage_roofline", "roofline"):
        if d.get(k):
            print(f"   {k}: {d[k]}")
    print(f"   stdout: {d['config'].get('stdout')!r}")
