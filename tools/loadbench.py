#!/usr/bin/env python3
"""Host -> HBM rate of the loader: qe_load_relation from pageable host
columns (numpy arrays, as the reference's read_relations would hand them over; the drop-in
`queries` binary passes mmap'd file columns the same way), then one C3 query on the loaded
relations so the PCIe-inclusive rate of the whole job can be stated.

    python tools/loadbench.py [--rows 100000000] [--reps 2]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "query-compiler-executor_amd"))

from qe import datagen as dg  # noqa: E402
from qe import lib  # noqa: E402

QUERY = "0 1 2 3|0.1=1.0&1.1=2.0&2.1=3.0&3.2>1000000000&3.2<3000000000|1.2 2.2 3.2\n"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=100_000_000)
    ap.add_argument("--reps", type=int, default=2)
    a = ap.parse_args()
    import torch
    torch.cuda.init()
    n = a.rows
    t = time.time()
    host = []
    for r in range(4):
        host.append([dg.column(1, r, c, n, k) for c, k in enumerate([("mod", n), ("mod", n), ("hi32",)])])
        print(f"[load] relation {r} generated on the host", file=sys.stderr, flush=True)
    print(f"[load] generated 4 x {n} x 3 host columns in {time.time() - t:.1f}s", file=sys.stderr)
    out = {}
    for rep in range(a.reps):
        ctx = lib.Ctx(0)
        t = time.time()
        for cols in host:
            ctx.load_relation(cols)
        ctx.sync()
        wall = time.time() - t
        s, b = ctx.load_stats()
        t = time.time()
        res, rc = ctx.run(QUERY)
        q = time.time() - t
        rows = ctx.last_result_rows()
        out = {"bytes": b, "load_s": round(s, 4), "load_GBps": round(b / s / 1e9, 2), "wall_s": round(wall, 4),
               "query_s": round(q, 4), "result_rows": rows,
               "host_inclusive_tuples_per_s": round(rows / (wall + q), 1), "stdout": res}
        print(json.dumps(out), flush=True)
        ctx.close()


if __name__ == "__main__":
    main()
