#!/usr/bin/env python3
"""Kernel-level timing of libqe primitives at full size (tuning aid, not the headline bench).

    python tools/kbench.py [sort|merge|payloads|all] [--n 100000000] [--reps 5]
Prints per-kernel ms (HIP events on the libqe stream) and algorithmic GB/s.
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "query-compiler-executor_amd"))

from qe import lib  # noqa: E402


def report(ctx, label, reps):
    st = ctx.kernel_stats()
    tot = 0.0
    for k, s in sorted(st.items(), key=lambda kv: -kv[1]["ms"]):
        if not s["launches"]:
            continue
        ms = s["ms"] / reps
        tot += ms
        gbs = s["alg_bytes"] / (s["ms"] * 1e-3) / 1e9 if s["ms"] else 0
        print(f"  {label:10s} {k:22s} {ms:8.3f} ms/rep  {s['launches'] / reps:5.1f} launches  {gbs:8.1f} GB/s")
    print(f"  {label:10s} {'TOTAL':22s} {tot:8.3f} ms/rep", flush=True)
    ctx.reset_stats()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("what", nargs="?", default="all")
    ap.add_argument("--n", type=int, default=100_000_000)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    import torch
    torch.cuda.init()          # torch's HIP runtime first (as bench.py and the tests do)
    ctx = lib.Ctx(0)
    n = a.n
    kinds = [("mod", n), ("mod", n), ("hi32",)]
    r0 = ctx.gen_relation(n, kinds, seed=1, gen_rel=0)
    r1 = ctx.gen_relation(n, kinds, seed=1, gen_rel=1)
    ctx.sync()
    ctx.set_profiling(True)
    if a.what in ("sort", "all"):
        for rep in range(a.reps + 1):
            p = ctx.gather_pairs(ctx.column(r0, 1), None)
            ctx.sort_pairs(p)
            ctx.pairs_free(p)
            if rep == 0:
                ctx.reset_stats()
        report(ctx, f"sort{os.environ.get('QE_SORT_MAXBITS', '')}", a.reps)
    if a.what in ("merge", "all"):
        R = ctx.gather_pairs(ctx.column(r0, 1), None)
        S = ctx.gather_pairs(ctx.column(r1, 0), None)
        ctx.sort_pairs(R)
        ctx.sort_pairs(S)
        ctx.reset_stats()
        for rep in range(a.reps):
            x, y = ctx.merge_join(R, S)
            ctx.list_free(x)
            ctx.list_free(y)
        report(ctx, "merge", a.reps)
    if a.what in ("filter", "all"):
        col = ctx.column(r0, 2)   # hi32: uniform in [0, 2^32)
        for rep in range(a.reps):
            l1 = ctx.filter_scan(col, ">", 1_000_000_000)
            ctx.filter_refine(col, "<", 3_000_000_000, l1)
            ctx.list_free(l1)
        report(ctx, "filter", a.reps)
    if a.what in ("bucket", "all"):
        # the N-rank plan's local bucket of a replicated column: nparts x n rows scanned
        parts = int(os.environ.get("QE_KB_PARTS", "8"))
        big = ctx.gen_relation(n * parts, [("mod", n * parts)], seed=1, gen_rel=5)
        ctx.sync()
        ctx.reset_stats()
        for rep in range(a.reps):
            p = ctx.bucket_select(ctx.column(big, 0), parts, rep % parts)
            ctx.pairs_free(p)
        report(ctx, "bucket", a.reps)
    if a.what in ("partition", "all"):
        import torch
        parts = int(os.environ.get("QE_KB_PARTS", "8"))
        c = ctx.column(r0, 1)
        cols = [torch.empty(n, dtype=torch.int32, device="cuda") for _ in range(2)]
        ok = torch.empty(n, dtype=torch.int64, device="cuda")
        oc = [torch.empty(n, dtype=torch.int32, device="cuda") for _ in range(2)]
        torch.cuda.synchronize()
        ctx.reset_stats()
        for rep in range(a.reps):
            ctx.partition(c.d, n, [t.data_ptr() for t in cols], parts, ok.data_ptr(), [t.data_ptr() for t in oc])
        report(ctx, "partition", a.reps)
    if a.what in ("gather", "all"):
        R = ctx.gather_pairs(ctx.column(r0, 1), None)
        ctx.sort_pairs(R)
        rows = lib.List()
        ctx.is_sorted(R)           # completes a deferred sort before its rowids are read directly
        rows.d, rows.n, rows.cap = R.val, R.n, R.n
        for rep in range(a.reps):
            p = ctx.gather_pairs(ctx.column(r1, 1), rows)
            ctx.pairs_free(p)
        report(ctx, "gather", a.reps)
    ctx.close()


if __name__ == "__main__":
    main()
