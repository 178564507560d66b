#!/usr/bin/env python3
"""Phase timing of mj_fused / radix_pass_kernel tiles from a -DQE_DIAG_STAMPS build (tuning aid).

    QE_LIB_PATH=.../build/diag/libqe_STAMPS.so python tools/stamps.py [--n 100000000]
Each tile's thread 0 stamps s_memrealtime (100 MHz) after every barrier-separated phase; this
prints the mean duration of each phase, the launch span and the mean number of tiles in flight.
"""
import argparse
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "query-compiler-executor_amd"))

from qe import lib  # noqa: E402

SLOTS = 8
PHASES = {
    "mj": ["ticket+win", "stage", "walk+annot+scan", "lookback+flags", "emit"],
    "sort": ["ticket+zero", "load+rank", "totals+publish+scan", "stage+lookback(t0)", "lookback wait", "write"],
    "cp": ["ticket", "load+ballots", "scan+lookback", "stage", "write"],
    "ag": ["load+keys", "walks", "sums"],
    "cpp": ["ballots (data wait)", "scan+publish", "stage+prefetch+lookback", "write"],
    "ws": ["ticket", "loads+ballots", "lookback", "stores"],
    "wsp": ["lookback (next loads in flight)", "stores"],
    "hj": ["bounds+loads issued", "R loaded+hist", "scan+scatter", "S counts+wave scans", "slice atomic", "emit (t0)"],
    "hjc": ["bounds+loads issued+head init", "R chained (loads landed)", "S counts+wave scans", "slice atomic", "emit (t0)"],
    "p2": ["zero+loads issued", "rank (loads landed)", "digit scan", "stage+payload loads", "words out", "payloads out"],
}


def report(ctx, which, ntiles):
    buf = np.zeros(ntiles * SLOTS, dtype=np.uint64)
    fn = ctx.lib.qe_diag_stamps
    fn.argtypes = [C.c_char_p, C.c_void_p, C.c_uint64]
    src = "cp" if which in ("cpp", "ws", "wsp") else "sort" if which == "p2" else "hj" if which == "hjc" else which
    rc = fn(src.encode(), buf.ctypes.data, buf.size)   # "hj", "p2": the sort file
    assert rc == 0, rc
    st = buf.reshape(ntiles, SLOTS).astype(np.int64)
    names = PHASES[which]
    k = len(names) + 1
    st = st[:, :k]
    ok = (st > 0).all(axis=1)
    st = st[ok]
    if not len(st):   # (a kernel form that does not stamp every phase)
        print(f"== {which}: no tile with all {k} stamps")
        return
    d = np.diff(st, axis=1) * 10.0 / 1000.0   # ticks of 10 ns -> us
    span = (st[:, -1].max() - st[:, 0].min()) * 10.0 / 1000.0
    busy = (st[:, -1] - st[:, 0]).sum() * 10.0 / 1000.0
    if which in ("ws", "wsp"):   # start/end order: how far behind its dispatch a tile's lookback resolves
        order = np.argsort(st[:, 0])
        print(f"   start spread {np.ptp(st[:, 0]) * 0.01:.1f} us; tiles ordered by start finish "
              f"{np.mean(np.diff(st[order, -1]) < 0) * 100:.1f}% out of order")
    print(f"== {which}: {ok.sum()} tiles, span {span:.1f} us, mean tiles in flight {busy / span:.1f}, "
          f"mean tile {(st[:, -1] - st[:, 0]).mean() * 0.01:.2f} us")
    for i, nm in enumerate(names):
        col = d[:, i]
        print(f"   {nm:24s} mean {col.mean():8.3f} us  p50 {np.median(col):8.3f}  p99 {np.percentile(col, 99):8.3f}")


def report_split(ctx, ntiles):
    """mj only: thread 0's walk end (slot 6) and annotate end (slot 7) inside phase 2->3"""
    buf = np.zeros(ntiles * SLOTS, dtype=np.uint64)
    ctx.lib.qe_diag_stamps(b"mj", buf.ctypes.data, buf.size)
    st = buf.reshape(ntiles, SLOTS).astype(np.int64)
    ok = (st[:, [2, 6, 7, 3]] > 0).all(axis=1)
    st = st[ok]
    for nm, x, y in (("walk (t0)", 2, 6), ("annotate (t0)", 6, 7), ("block scan barrier", 7, 3)):
        d = (st[:, y] - st[:, x]) * 0.01
        print(f"   {nm:24s} mean {d.mean():8.3f} us  p50 {np.median(d):8.3f}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=100_000_000)
    ap.add_argument("--what", default="sort,mj")
    ap.add_argument("--cp-tile", type=int, default=8192, help="compact tile rows (CB x FS_ITEMS x 2)")
    a = ap.parse_args()
    ctx = lib.Ctx(0)
    n = a.n
    if "ag" in a.what:   # the aggregate join's tile kernel on C5-shaped data (first 65536 tiles)
        from qe import datagen as dg
        dg.gen_c5(ctx, n)
        ctx.run(dg.C5_QUERY)
        report(ctx, "ag", min(65536, (2 * n + 4095) // 4096))
        ctx.close()
        return
    if a.what in ("c3p1", "c3p2"):
        # one selected first / second pass of the C3 plan's two-level sorts: QE_STAMP_SEL=p1:K / p2:K
        # must be set in the environment (the launches are numbered on stderr); the query runs once
        kinds = [("mod", n), ("mod", n), ("hi32",)]
        for r in range(4):
            ctx.gen_relation(n, kinds, seed=1, gen_rel=r)
        ctx.sync()
        q = "0 1 2 3|0.1=1.0&1.1=2.0&2.1=3.0&3.2>1000000000&3.2<3000000000|1.2 2.2 3.2\n"
        ctx.run_dist(q, None)
        ctx.sync()
        report(ctx, "sort" if a.what == "c3p1" else "p2", 65536)
        ctx.close()
        return
    if "hj" in a.what:   # the bucket join of the last C3 join (the partitioned plan at N = 1)
        kinds = [("mod", n), ("mod", n), ("hi32",)]
        for r in range(4):
            ctx.gen_relation(n, kinds, seed=1, gen_rel=r)
        ctx.sync()
        q = "0 1 2 3|0.1=1.0&1.1=2.0&2.1=3.0&3.2>1000000000&3.2<3000000000|1.2 2.2 3.2\n"
        for _ in range(2):
            ctx.run_dist(q, None)
        ctx.sync()
        report(ctx, "hjc" if os.environ.get("QE_HJ_CHAIN", "1") != "0" else "hj", 32768)
        ctx.close()
        return
    kinds = [("mod", n), ("mod", n), ("hi32",)]
    r0 = ctx.gen_relation(n, kinds, seed=1, gen_rel=0)
    r1 = ctx.gen_relation(n, kinds, seed=1, gen_rel=1)
    if "cp" in a.what:
        l1 = ctx.filter_scan(ctx.column(r0, 2), ">", 1_000_000_000)
        ctx.sync()
        if os.environ.get("QE_WSCAN", "1") != "0" and os.environ.get("QE_WSPIPE", "1") != "0":
            report(ctx, "wsp", (n + 1023) // 1024)             # persistent wave tiles of 16 x 64 rows
        elif os.environ.get("QE_WSCAN", "1") != "0":           # wave tiles of WS_STEPS x 64 rows
            report(ctx, "ws", (n + 2047) // 2048)
        else:
            report(ctx, "cpp" if os.environ.get("QE_CP_PIPE", "1") != "0" else "cp", (n + a.cp_tile - 1) // a.cp_tile)
        ctx.list_free(l1)
    if "sort" not in a.what and "mj" not in a.what:
        ctx.close()
        return
    R = ctx.gather_pairs(ctx.column(r0, 1), None)
    S = ctx.gather_pairs(ctx.column(r1, 0), None)
    ctx.sort_pairs(R)
    ctx.sort_pairs(S)
    ctx.sync()
    report(ctx, "sort", (n + 8191) // 8192)   # last pass of S's sort
    for _ in range(2):
        x, y = ctx.merge_join(R, S)
        ctx.sync()
        ctx.list_free(x)
        ctx.list_free(y)
    report(ctx, "mj", (n + 2047) // 2048)
    report_split(ctx, (n + 2047) // 2048)
    ctx.close()


if __name__ == "__main__":
    main()
