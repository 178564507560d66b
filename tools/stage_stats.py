#!/usr/bin/env python3
"""rocprofv3 --kernel-trace --stats summary -> bench.py stage names (per-launch average), so the
profile can be checked against the bench line's HIP-event numbers.

    python tools/stage_stats.py gpurun_out/TAG_trace/run_kernel_stats.csv --out profiles/...json
"""
import argparse
import csv
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_traffic import stage_of  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("stats_csv")
    ap.add_argument("--out")
    ap.add_argument("--command", default="")
    ap.add_argument("--workload", default="c3")
    a = ap.parse_args()
    acc = defaultdict(lambda: [0, 0.0])
    with open(a.stats_csv) as f:
        for row in csv.DictReader(f):
            st = stage_of(row["Name"], a.workload) or row["Name"].split("(")[0][:60]
            acc[st][0] += int(row["Calls"])
            acc[st][1] += float(row["TotalDurationNs"])
    doc = {"command": a.command, "source": a.stats_csv, "workload": a.workload,
           "stages": {k: {"calls": c, "total_ms": round(t / 1e6, 3), "avg_ms": round(t / 1e6 / c, 4)}
                      for k, (c, t) in sorted(acc.items(), key=lambda kv: -kv[1][1])}}
    for k, v in doc["stages"].items():
        print(f"{k:28s} {v['calls']:6d} calls {v['total_ms']:10.3f} ms  avg {v['avg_ms']:.4f} ms")
    if a.out:
        with open(a.out, "w") as fo:
            json.dump(doc, fo, indent=1)


if __name__ == "__main__":
    main()
