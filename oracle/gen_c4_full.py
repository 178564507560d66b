#!/usr/bin/env python3
"""Generate tests/golden/full/c4_full.json: the C4 batch at FULL size, expected output by
oracle/cpu_ref.  TEST INFRASTRUCTURE ONLY (the checker, never the thing measured).

    make -C oracle cpuref && python oracle/gen_c4_full.py [--workers 8]

The rand-invariance gate (oracle/gen_golden.py) ran the real reference binary on the C4 queries
at N/100 (tests/golden/c4.json: 874 deterministic queries).  At full size (qe.datagen.c4_spec(1.0):
14 relations of 1e5..1e7 rows) the reference itself is too slow to run (its hashmap dedup,
src/join.c:362-367, is O(pairs * bucket length)), so the oracle is cpu_ref -- the C restatement
pinned byte for byte on every golden of the real binary (tests/test_oracle.py).  Each query runs
on its own (cpu_ref keeps no state between queries; the reference's only cross-query state is
rand(), which the gate excludes).  The fixture holds the dataset spec, the query text and the
expected stdout bytes -- no relation data (the GPU test generates the relations in HBM with the
same splitmix64 generator).
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import multiprocessing as mp
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(ROOT, "query-compiler-executor_amd"))

from qe import datagen as dg  # noqa: E402

SO = os.path.join(HERE, "build", "libcpuref.so")
OUT = os.path.join(ROOT, "tests", "golden", "full", "c4_full.json")

_H = {}


def _setup():
    lib = C.CDLL(SO)
    lib.cpuref_create.restype = C.c_void_p
    lib.cpuref_add_relation.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64, C.POINTER(C.c_void_p)]
    lib.cpuref_run_str.argtypes = [C.c_void_p, C.c_char_p, C.POINTER(C.c_void_p), C.POINTER(C.c_size_t)]
    specs = dg.c4_spec(1.0)
    rels = dg.make_relations(specs, dg.C4_SEED)
    h = lib.cpuref_create()
    keep = []
    for sp, cols in zip(specs, rels):
        arr = (C.c_void_p * len(cols))(*[c.ctypes.data for c in cols])
        keep.append(arr)
        lib.cpuref_add_relation(h, sp.rows, len(cols), arr)
    _H.update(lib=lib, h=h, keep=keep, rels=rels, specs=specs)


def _run(q: str):
    lib, h = _H["lib"], _H["h"]
    out, n = C.c_void_p(), C.c_size_t()
    t0 = time.perf_counter()
    rc = lib.cpuref_run_str(h, q.encode(), C.byref(out), C.byref(n))
    return C.string_at(out, n.value).decode("latin-1"), rc, time.perf_counter() - t0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workers", type=int, default=min(8, os.cpu_count() or 1))
    a = ap.parse_args()
    with open(os.path.join(ROOT, "tests", "golden", "c4.json")) as f:
        small = json.load(f)
    queries = [c["input"] for c in small["cases"] if c["rc"] == 0]
    _setup()                                   # relations built once, shared by fork
    t0 = time.time()
    with mp.get_context("fork").Pool(a.workers) as pool:
        res = pool.map(_run, queries, chunksize=4)
    specs = _H["specs"]
    doc = {
        "name": "c4_full",
        "oracle": "oracle/cpu_ref (pinned to the real reference on every golden; tests/test_oracle.py)",
        "generator": "qe.datagen.c4_spec(1.0), splitmix64 (SURVEY.md §9.1)",
        "script": "oracle/gen_c4_full.py",
        "dataset": {"seed": dg.C4_SEED,
                    "relations": [{"rows": s.rows, "kinds": [list(k) for k in s.kinds]} for s in specs]},
        "cpu_seconds": round(sum(r[2] for r in res), 2),
        "cases": [{"input": q, "stdout": o, "rc": rc} for q, (o, rc, _) in zip(queries, res)],
    }
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    with open(OUT, "w") as f:
        json.dump(doc, f, indent=0)
        f.write("\n")
    print(f"{len(queries)} queries, {doc['cpu_seconds']} s of cpu_ref in {time.time() - t0:.1f} s wall -> {OUT}")


if __name__ == "__main__":
    main()
