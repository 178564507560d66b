"""Key-partitioned multi-GPU execution of join queries.

One process per GPU (torch.distributed; backend "nccl" = RCCL over xGMI).  Every rank holds a
replica of the base columns and owns a contiguous rowid slice of every relation.  A query runs
as a relational plan over the device primitives of libqe:

  filters   -- each rank scans its own slice (qe_filter_scan_range); a second filter on the same
               binding refines it and prints the global count (all-reduce), as the reference's
               exec_filter_rel_exists does (src/filter.c:3-35)
  joins     -- both inputs are gathered to keys (replicated columns, local), hash-partitioned on
               the key (qe_partition: dest = hi32(mix(key)) * world >> 32), exchanged with one RCCL
               all-to-all per array, and joined locally (qe_join_indices: LSD radix sort + merge
               path); rowid columns of the intermediate ride along (qe_take_u32).  Columns no
               later predicate or select needs are dropped before the exchange.
  checksums -- local gather-sum (qe_checksum) + all-reduce of the uint64 sums (exact mod 2^64)

The plan computes relational semantics.  It equals the reference's output on the reference's
well-defined (rand-invariant, relational) domain -- every measured config (SURVEY.md §8(c)
item 3) -- and refuses shapes it does not cover (NotSupported) instead of guessing.  The
single-GPU drop-in for arbitrary queries is libqe's faithful executor (qe_run_queries).

The executor is engine-agnostic: GPUEngine drives libqe; tests/ supply a numpy engine to run the
same plan under world_size-2 gloo on CPU.
"""
from __future__ import annotations

import os
import re
import time
from dataclasses import dataclass

import numpy as np

M64 = (1 << 64) - 1


class NotSupported(Exception):
    pass


# ---------------------------------------------------------------------------------------------
# query model: the reference grammar (src/parsing.c) for well-formed lines, and the exact
# predicate arrangement of src/pred_arrange.c:50-93 (index-lag quirk included)
# ---------------------------------------------------------------------------------------------
@dataclass
class Pred:
    kind: str              # "join" | "filter"
    a: tuple               # (binding, column)
    b: tuple | None        # join: (binding, column); filter: None
    op: str
    const: int = 0

    def second(self):      # what is_match reads through `second`
        return self.b if self.kind == "join" else (self.const, 0)


def parse(line: str):
    rels_s, preds_s, sel_s = line.strip().split("|")
    rels = [int(x) for x in rels_s.split(" ")]
    preds = []
    for p in preds_s.split("&"):
        m = re.fullmatch(r"(\d+)\.(\d+)(.)(\d+)\.(\d+)", p)
        if m:
            a, b, op, c, d = m.groups()
            preds.append(Pred("join", (int(a), int(b)), (int(c), int(d)), op))
            continue
        m = re.fullmatch(r"(\d+)\.(\d+)(.)(\d+)", p)
        if not m:
            raise NotSupported(f"predicate {p!r}")
        a, b, op, c = m.groups()
        preds.append(Pred("filter", (int(a), int(b)), None, op, int(c) & 0xFFFFFFFF))
    sels = [tuple(int(v) for v in s.split(".")) for s in sel_s.split(" ")]
    return rels, preds, sels


def _is_match(l: Pred, r: Pred) -> bool:
    la, lb, ra, rb = l.a, l.second(), r.a, r.second()
    return la == ra or la == rb or lb == ra or lb == rb


def arrange(preds: list[Pred]) -> list[Pred]:
    p = list(preds)
    n = len(p)
    index = 0
    for i in range(1, n):                        # group_filters (p[0] never examined)
        if p[i].kind == "filter":
            s = i
            for _ in range(i - index):
                p[s], p[s - 1] = p[s - 1], p[s]
                s -= 1
            index += 1
    i = index
    while i < n - 1:                             # group_matches, `current` aliases slot i
        swapped = False
        for j in range(i + 1, n):
            if _is_match(p[i], p[j]):
                index += 1
                p[index], p[j] = p[j], p[index]
                swapped = True
        i = index if swapped else i + 1
    return p


def owned_range(rows: int, rank: int, world: int) -> tuple[int, int]:
    return rows * rank // world, rows * (rank + 1) // world


# ---------------------------------------------------------------------------------------------
# GPU engine (libqe + torch.distributed)
# ---------------------------------------------------------------------------------------------
class DArr:
    """A device array: pointer + length + the object that owns the memory."""

    __slots__ = ("ptr", "n", "keep", "free", "bits")

    def __init__(self, ptr, n, keep=None, free=None, bits=None):
        # bits: (OR, AND) bounds of the keys (the source column's statistics: a subset of a
        # column varies in no bit the column does not), so the sort skips its reduction pass
        self.ptr, self.n, self.keep, self.free, self.bits = ptr, n, keep, free, bits

    def __del__(self):
        if self.free is not None:
            try:
                self.free()
            except Exception:
                pass


class GPUEngine:
    def __init__(self, ctx, rank: int, world: int, group=None):
        import torch
        import torch.distributed as dist
        self.torch, self.dist = torch, dist
        self.ctx, self.rank, self.world, self.group = ctx, rank, world, group
        self.comm_dev = "cpu"
        if world > 1 and dist.get_backend(group) == "nccl":
            self.comm_dev = f"cuda:{torch.cuda.current_device()}"
        from . import lib
        self.lib = lib

    # -- ownership helpers
    def _list(self, l):
        ctx = self.ctx
        return DArr(l.d, l.n, keep=l, free=lambda: ctx.list_free(l))

    def _as_list(self, a: DArr):
        l = self.lib.List()
        l.d, l.n, l.cap, l.flags = a.ptr, a.n, a.n, 0
        return l

    def length(self, a: DArr) -> int:
        return a.n

    def scan(self, rel, col, start, end, op, v) -> DArr:
        return self._list(self.ctx.filter_scan_range(self.ctx.column(rel, col), start, end, op, v))

    def iota(self, start, n) -> DArr:
        return self._list(self.ctx.iota(start, n))

    def refine(self, rel, col, rows: DArr, op, v) -> DArr:
        """order-preserving refinement of a list this plan owns alone (updated in place)"""
        l = rows.keep
        if not isinstance(l, self.lib.List):
            raise NotSupported("refine of a borrowed list")
        self.ctx.filter_refine(self.ctx.column(rel, col), op, v, l)
        rows.ptr, rows.n = l.d, l.n
        return rows

    def keys(self, rel, col, rows: DArr) -> DArr:
        p = self.ctx.gather_pairs(self.ctx.column(rel, col), self._as_list(rows))
        ctx = self.ctx
        return DArr(p.key, p.n, keep=p, free=lambda: ctx.pairs_free(p), bits=self.ctx.column_bits(rel, col))

    def filter_idx(self, rel, col, rows: DArr, op, v) -> DArr:
        k = self.keys(rel, col, rows)
        c = self.lib.Col()
        c.d, c.n = k.ptr, k.n
        out = self._list(self.ctx.filter_scan(c, op, v))
        del k
        return out

    def take(self, rows: DArr, idx: DArr) -> DArr:
        return self._list(self.ctx.take_u32(rows.ptr, self._as_list(idx)))

    def join_local(self, ka: DArr, kb: DArr):
        ia, ib = self.ctx.join_indices(ka.ptr, ka.n, kb.ptr, kb.n)
        return self._list(ia), self._list(ib)

    def base_side(self, rel, col):
        """a whole base relation as a join side: (keys, rowids or None = row i).  One rank: the
        column itself (zero copy).  N ranks: the local hash bucket of the replicated column
        (qe_bucket_select) -- the rows the exchange would deliver, without moving them."""
        c = self.ctx.column(rel, col)
        if self.world == 1:
            return DArr(c.d, c.n, bits=self.ctx.column_bits(rel, col)), None
        p = self.ctx.bucket_select(c, self.world, self.rank)
        ctx = self.ctx
        keys = DArr(p.key, p.n, keep=p, free=lambda: ctx.pairs_free(p), bits=self.ctx.column_bits(rel, col))
        return keys, DArr(p.val, p.n, keep=keys)

    def base_side_light(self, rel, col, heavy):
        """base_side without the heavy keys (skew path): the local bucket minus heavy keys"""
        if self.world == 1 and len(heavy) == 0:
            return self.base_side(rel, col)
        p = self.ctx.bucket_select(self.ctx.column(rel, col), self.world, self.rank, heavy)
        ctx = self.ctx
        keys = DArr(p.key, p.n, keep=p, free=lambda: ctx.pairs_free(p), bits=self.ctx.column_bits(rel, col))
        return keys, DArr(p.val, p.n, keep=keys)

    def join_count_sums(self, ka: DArr, va, kb: DArr, vb, sel_a: list, sel_b: list):
        """aggregate form of the merge (no pair materialised): (pairs, [sum over pairs of
        col[rowid_A] for (rel, col) in sel_a], [... sel_b]) mod 2^64 -- qe_merge_join_counts +
        qe_checksum_weighted"""
        P = self.lib.Pairs
        sides = []
        for k, v in ((ka, va), (kb, vb)):
            p = P()
            p.key, p.val, p.n, p.flags, p.owns = k.ptr, (v.ptr if v is not None else None), k.n, 0, 0
            if k.bits is not None:
                p.kor, p.kand, p.flags = k.bits[0], k.bits[1], 4          # QE_PAIRS_BITS
            sides.append(p)
        A, B = sides
        try:
            self.ctx.sort_pairs(A)
            self.ctx.sort_pairs(B)
            pairs = self.ctx.merge_join_counts(A, B)
            sa = [self.ctx.checksum_weighted(self.ctx.column(r, c), A) for (r, c) in sel_a]
            sb = [self.ctx.checksum_weighted(self.ctx.column(r, c), B) for (r, c) in sel_b]
        finally:
            self.ctx.pairs_free(A)
            self.ctx.pairs_free(B)
        return pairs, sa, sb

    def heavy_stats(self, rel, col, start, end, heavy, val=None, weights=None):
        v = self.ctx.column(*val) if val is not None else None
        return self.ctx.heavy_stats(self.ctx.column(rel, col), start, end, heavy, v, weights)

    def column_prefix(self, rel, col, m):
        c = self.ctx.column(rel, col)
        p = self.lib.Pairs()
        p.key, p.val, p.match, p.n = c.d, None, None, min(m, c.n)
        out = np.empty(p.n, dtype=np.uint64)
        self.ctx._chk(self.ctx.lib.qe_pairs_to_host(self.ctx.h, self.lib.C.byref(p), out.ctypes.data, None))
        return out

    def allreduce_vec(self, a: np.ndarray) -> np.ndarray:
        a = np.ascontiguousarray(a, dtype=np.uint64)
        if self.world == 1 or a.size == 0:
            return a
        t = self.torch.from_numpy(a.view(np.int64).copy()).to(self.comm_dev)
        self.dist.all_reduce(t, group=self.group)
        return t.cpu().numpy().view(np.uint64)

    def join_pairs(self, ka: DArr, va, kb: DArr, vb):
        """sort both sides by key (stable LSD radix) and merge: aligned outputs, va[i] (or i when
        va is None) for side A and likewise for B, in key order"""
        P = self.lib.Pairs
        sides = []
        for k, v in ((ka, va), (kb, vb)):
            p = P()
            p.key, p.val, p.n, p.flags, p.owns = k.ptr, (v.ptr if v is not None else None), k.n, 0, 0
            if k.bits is not None:
                p.kor, p.kand, p.flags = k.bits[0], k.bits[1], 4          # QE_PAIRS_BITS: column stats
            sides.append(p)
        A, B = sides
        try:
            self.ctx.sort_pairs(A)
            self.ctx.sort_pairs(B)
            oa, ob = self.ctx.merge_join(A, B)
        finally:
            self.ctx.pairs_free(A)
            self.ctx.pairs_free(B)
        return self._list(oa), self._list(ob)

    def keep_equal(self, ka: DArr, kb: DArr) -> DArr:
        P = self.lib.Pairs
        A, B = P(), P()
        A.key, A.n, A.flags = ka.ptr, ka.n, 1
        B.key, B.n, B.flags = kb.ptr, kb.n, 1
        a, b = self.ctx.scan_join(A, B)
        self.ctx.list_free(b)
        return self._list(a)

    def checksum(self, rel, col, rows: DArr) -> int:
        return self.ctx.checksum(self.ctx.column(rel, col), self._as_list(rows))

    def allreduce(self, x: int) -> int:
        if self.world == 1:
            return x & M64
        t = self.torch.tensor([x - (1 << 64) if x >= (1 << 63) else x], dtype=self.torch.int64,
                              device=self.comm_dev)
        self.dist.all_reduce(t, group=self.group)
        return int(t.item()) & M64

    def exchange(self, keys: DArr, cols: list[DArr]):
        """hash-partition rows on keys and all-to-all them; returns this rank's bucket"""
        return self.exchange_finish(self.exchange_start(keys, cols))

    def exchange_start(self, keys: DArr, cols: list[DArr]):
        """partition (libqe stream) + the counts all-to-all, then the data all-to-alls queued
        asynchronously on the communicator's stream: the caller overlaps its next libqe work
        (the other join side) with the transfer and calls exchange_finish"""
        torch, dist, W = self.torch, self.dist, self.world
        n = keys.n
        dev = f"cuda:{torch.cuda.current_device()}"
        sk = torch.empty(max(1, n), dtype=torch.int64, device=dev)
        sc = [torch.empty(max(1, n), dtype=torch.int32, device=dev) for _ in cols]
        torch.cuda.synchronize()
        counts = self.ctx.partition(keys.ptr, n, [c.ptr for c in cols], W, sk.data_ptr(),
                                    [t.data_ptr() for t in sc])   # synchronises the libqe stream
        cnt = torch.tensor(counts, dtype=torch.int64, device=self.comm_dev)
        rcnt = torch.empty_like(cnt)
        dist.all_to_all_single(rcnt, cnt, group=self.group)
        out_splits = [int(v) for v in rcnt.tolist()]
        total = sum(out_splits)
        outs, works, keep = [], [], [sk, sc]
        for src, dt in [(sk, torch.int64)] + [(t, torch.int32) for t in sc]:
            s = src[:n].to(self.comm_dev) if self.comm_dev != dev else src[:n]
            r = torch.empty(max(1, total), dtype=dt, device=self.comm_dev)
            works.append(dist.all_to_all_single(r[:total], s, out_splits, counts, group=self.group, async_op=True))
            keep.append(s)
            outs.append(r)
        return (outs, works, keep, total, dev, keys.bits)

    def exchange_finish(self, h):
        outs, works, keep, total, dev, bits = h
        for w in works:
            w.wait()
        if self.comm_dev != dev:
            outs = [r.to(dev) for r in outs]
        self.torch.cuda.synchronize()
        del keep
        rk = DArr(outs[0].data_ptr(), total, keep=outs[0], bits=bits)
        rc = [DArr(t.data_ptr(), total, keep=t) for t in outs[1:]]
        return rk, rc


# ---------------------------------------------------------------------------------------------
# the plan
# ---------------------------------------------------------------------------------------------
class DistExecutor:
    """Runs one query line with the key-partitioned relational plan on `engine`.

    Components: bindings already joined together, each {binding: rowid list}; a whole base
    relation not touched by any filter or join yet is {binding: None} and is never materialised
    (as a join side it is the column itself on one rank, the local hash bucket of the
    replicated column on N ranks).  Consecutive joins are reordered greedily (smallest
    |A| + |B| first, global sizes) -- relational semantics do not depend on the order, and
    filters, whose stray count lines do, keep their place between the runs of joins."""

    def __init__(self, engine, rel_rows: list[int], reorder: bool | None = None):
        self.e = engine
        self.rel_rows = rel_rows
        self.reorder = (os.environ.get("QE_DIST_REORDER", "1") != "0") if reorder is None else reorder

    def _base(self, rel):
        s, t = owned_range(self.rel_rows[rel], self.e.rank, self.e.world)
        return self.e.iota(s, t - s)

    def run(self, line: str):
        """-> (stdout text, global result rows)"""
        e = self.e
        rels, preds, sels = parse(line)
        preds = arrange(preds)
        nb = len(rels)
        for p in preds:
            for (b, c) in [p.a] + ([p.b] if p.b else []):
                if b >= nb or rels[b] >= len(self.rel_rows):
                    raise NotSupported("binding out of range")
            if p.kind == "join" and rels[p.a[0]] == rels[p.b[0]] and p.a[1] == p.b[1]:
                raise NotSupported("same relation and column on both sides (reference DO_NOTHING)")
            if p.kind == "filter" and p.op not in "=<>":
                raise NotSupported("operator")
        joined = {b for p in preds if p.kind == "join" for b in (p.a[0], p.b[0])}
        for (b, _) in sels:
            if b not in joined:
                raise NotSupported("selected binding outside the join graph")
        out = []
        comp_of: dict[int, int] = {}            # binding -> component id
        comps: dict[int, dict] = {}             # component -> {binding: rowids | None (whole base)}
        size: dict[int, int] = {}               # component -> global rows
        lists: dict[int, object] = {}           # filtered, not yet joined bindings
        list_size: dict[int, int] = {}

        def need_of(pending):
            need = {b for (b, _) in sels}
            for q in pending:
                need.add(q.a[0])
                if q.b:
                    need.add(q.b[0])
            return need

        def component(b):
            if b in comp_of:
                return comp_of[b]
            cid = len(comps) + 1000 * (b + 1)
            if b in lists:
                comps[cid] = {b: lists.pop(b)}
                size[cid] = list_size.pop(b)
            else:
                comps[cid] = {b: None}
                size[cid] = self.rel_rows[rels[b]]
            comp_of[b] = cid
            return cid

        def rows_of(cid, b):
            if comps[cid][b] is None:
                comps[cid][b] = self._base(rels[b])
            return comps[cid][b]

        def side(cid, b, c, need):
            """start one join side; returns a function giving (keys, vals, carried), carried =
            [(binding, rowids | 'vals')].  An exchange is in flight between the two calls."""
            cols = comps[cid]
            if len(cols) == 1 and b in cols and cols[b] is None:
                keys, vals = e.base_side(rels[b], c)
                return lambda: (keys, vals, ([(b, "vals")] if b in need else []))
            keys = e.keys(rels[b], c, rows_of(cid, b))
            keep = [x for x in sorted(cols) if x in need]

            def done(keys, cur):
                if len(keep) == 1:
                    return keys, cur[keep[0]], [(keep[0], "vals")]
                return keys, None, [(x, cur[x]) for x in keep]
            if e.world > 1:
                if len(keep) > 4:
                    raise NotSupported("more than 4 rowid columns in one exchange")
                h = e.exchange_start(keys, [rows_of(cid, x) for x in keep])

                def finish():
                    rk, rc = e.exchange_finish(h)
                    return done(rk, dict(zip(keep, rc)))
                return finish
            cur = {x: rows_of(cid, x) for x in keep}
            return lambda: done(keys, cur)

        def do_join(p, pending):
            (ba, ca), (bb, cb) = p.a, p.b
            A, B = component(ba), component(bb)
            need = need_of(pending)
            if A == B:
                cols = comps[A]
                idx = e.keep_equal(e.keys(rels[ba], ca, rows_of(A, ba)), e.keys(rels[bb], cb, rows_of(A, bb)))
                comps[A] = {x: e.take(rows_of(A, x), idx) for x in list(cols)}
                size[A] = e.allreduce(e.length(idx))
                return
            # derived sides first, so their exchanges overlap the base side's local bucket scan
            A_base = len(comps[A]) == 1 and comps[A].get(ba, 0) is None
            if A_base:
                fb = side(B, bb, cb, need)
                fa = side(A, ba, ca, need)
            else:
                fa = side(A, ba, ca, need)
                fb = side(B, bb, cb, need)
            ka, va, carry_a = fa()
            kb, vb, carry_b = fb()
            oa, ob = e.join_pairs(ka, va, kb, vb)
            del ka, kb, va, vb
            merged = {}
            for carry, o in ((carry_a, oa), (carry_b, ob)):
                for x, r in carry:
                    merged[x] = o if isinstance(r, str) else e.take(r, o)
            if not merged:                       # nothing needed later: keep the row count
                merged[ba] = oa
            del comps[A], comps[B]
            comps[A] = merged
            size.pop(B, None)
            for x in list(comp_of):
                if comp_of[x] in (A, B):
                    comp_of[x] = A
            for x in merged:
                comp_of[x] = A
            size[A] = e.allreduce(e.length(next(iter(merged.values()))))

        def cost(p):
            A = comp_of.get(p.a[0])
            B = comp_of.get(p.b[0])
            if A is not None and A == B:
                return -1
            def sz(b, cid):
                if cid is not None:
                    return size[cid]
                return list_size[b] if b in lists else self.rel_rows[rels[b]]
            return sz(p.a[0], A) + sz(p.b[0], B)

        k = 0
        while k < len(preds):
            p = preds[k]
            if p.kind == "filter":
                b, c = p.a
                rel = rels[b]
                if b in comp_of:
                    cid = comp_of[b]
                    idx = e.filter_idx(rel, c, rows_of(cid, b), p.op, p.const)
                    comps[cid] = {bb: e.take(rows_of(cid, bb), idx) for bb in list(comps[cid])}
                    size[cid] = e.allreduce(e.length(idx))
                    out.append(f"{size[cid] & 0xFFFFFFFF:d}\n")
                elif b in lists:
                    lists[b] = e.refine(rel, c, lists[b], p.op, p.const)
                    list_size[b] = e.allreduce(e.length(lists[b]))
                    out.append(f"{list_size[b]:d}\n")
                else:
                    s_, t_ = owned_range(self.rel_rows[rel], e.rank, e.world)
                    lists[b] = e.scan(rel, c, s_, t_, p.op, p.const)
                    list_size[b] = e.allreduce(e.length(lists[b]))
                k += 1
                continue
            run_end = k
            while run_end < len(preds) and preds[run_end].kind == "join":
                run_end += 1
            run = preds[k:run_end]
            while run:
                j = min(range(len(run)), key=lambda i: (cost(run[i]), i)) if self.reorder else 0
                q = run.pop(j)
                do_join(q, run + preds[run_end:])
            k = run_end
        # print_sums
        roots = {comp_of[b] for (b, _) in sels}
        if len(roots) != 1:
            raise NotSupported("disconnected selects")
        cid = roots.pop()
        rows = size[cid]
        line_out = []
        for (b, c) in sels:
            s = e.allreduce(e.checksum(rels[b], c, rows_of(cid, b)))
            line_out.append("NULL " if rows == 0 else f"{s} ")
        out.append("".join(line_out) + "\n")
        return "".join(out), rows


# ---------------------------------------------------------------------------------------------
# the skewed 2-relation join in aggregate form (C5, SURVEY.md §8(e) "Skew")
# ---------------------------------------------------------------------------------------------
class DistAggJoin:
    """`r0 r1|0.a=1.b|sel...` (one equi-join, no filters) without materialising pairs, N ranks.

    sum over pairs of col(pR) = sum_k (sum_{r in R_k} col(r)) * |S_k| (and symmetrically), so:
      heavy keys -- the keys whose sampled frequency exceeds rows / (N * 64) on either side; the
                    sample is the first `sample` rows of the replicated key columns, identical on
                    every rank, so every rank derives the same list without communication.  Each
                    rank counts heavy keys over its own row slice of R and S (qe_heavy_stats),
                    the counts are all-reduced, and each rank adds
                    sum_{r in slice, key heavy} col(r) * |S_key| (weighted qe_heavy_stats) --
                    no heavy row moves and no rank holds a heavy key's whole run;
      light keys -- hash bucket per rank straight from the replicated columns
                    (qe_bucket_select, heavy keys left out), sorted, merged in aggregate form
                    (qe_merge_join_counts) and summed (qe_checksum_weighted);
    and the sums and pair counts are all-reduced (exact mod 2^64).  The line printed is the
    reference's print_sums line for the materialised join (SURVEY.md §9.5 proves the aggregate
    form equal to the reference at 20 k rows)."""

    def __init__(self, engine, rel_rows: list[int], sample: int = 1 << 21, heavy_div: int = 64):
        self.e, self.rel_rows, self.sample, self.heavy_div = engine, rel_rows, sample, heavy_div

    def heavy_keys(self, rel_a, ca, rel_b, cb) -> np.ndarray:
        e = self.e
        if e.world == 1:
            return np.zeros(0, np.uint64)
        out = set()
        for rel, c in ((rel_a, ca), (rel_b, cb)):
            pre = e.column_prefix(rel, c, self.sample)
            if pre.size == 0:
                continue
            u, cnt = np.unique(pre, return_counts=True)
            thr = pre.size / (e.world * self.heavy_div)
            out.update(u[cnt > thr].tolist())
        h = np.array(sorted(out), dtype=np.uint64)
        return h[:1024]

    def run(self, line: str):
        e = self.e
        rels, preds, sels = parse(line)
        joins = [p for p in preds if p.kind == "join"]
        if len(rels) != 2 or len(preds) != 1 or len(joins) != 1 or joins[0].a[0] == joins[0].b[0]:
            raise NotSupported("aggregate plan: exactly one join between two bindings, no filters")
        (ba, ca), (bb, cb) = joins[0].a, joins[0].b
        if rels[ba] == rels[bb] and ca == cb:
            raise NotSupported("same relation and column on both sides (reference DO_NOTHING)")
        ra, rb = rels[ba], rels[bb]
        sel_a = [(ra, c) for (b, c) in sels if b == ba]
        sel_b = [(rb, c) for (b, c) in sels if b == bb]
        heavy = self.heavy_keys(ra, ca, rb, cb)
        # light keys: local buckets, aggregate merge
        ka, va = e.base_side_light(ra, ca, heavy)
        kb, vb = e.base_side_light(rb, cb, heavy)
        pairs, sa, sb = e.join_count_sums(ka, va, kb, vb, sel_a, sel_b)
        del ka, kb, va, vb
        # heavy keys: slice counts -> global counts -> weighted slice sums
        if heavy.size:
            sa_, ta_ = owned_range(self.rel_rows[ra], e.rank, e.world)
            sb_, tb_ = owned_range(self.rel_rows[rb], e.rank, e.world)
            cA, _ = e.heavy_stats(ra, ca, sa_, ta_, heavy)
            cB, _ = e.heavy_stats(rb, cb, sb_, tb_, heavy)
            CA, CB = np.split(e.allreduce_vec(np.concatenate([cA, cB])), 2)
            sa = [(x + e.heavy_stats(ra, ca, sa_, ta_, heavy, val=sc, weights=CB)[1]) & M64
                  for x, sc in zip(sa, sel_a)]
            sb = [(x + e.heavy_stats(rb, cb, sb_, tb_, heavy, val=sc, weights=CA)[1]) & M64
                  for x, sc in zip(sb, sel_b)]
            heavy_pairs = sum(int(x) * int(y) for x, y in zip(CA.tolist(), CB.tolist()))
        else:
            heavy_pairs = 0
        red = e.allreduce_vec(np.array([pairs & M64] + sa + sb, dtype=np.uint64))
        total = int(red[0]) + heavy_pairs
        sums = {}
        for i, key in enumerate(sel_a):
            sums[("a", key)] = int(red[1 + i])
        for i, key in enumerate(sel_b):
            sums[("b", key)] = int(red[1 + len(sel_a) + i])
        parts = []
        for (b, c) in sels:
            s = sums[("a", (ra, c))] if b == ba else sums[("b", (rb, c))]
            parts.append("NULL " if total == 0 else f"{s} ")
        return "".join(parts) + "\n", total, int(heavy.size)


# ---------------------------------------------------------------------------------------------
# bench entry for N > 1 (launched by torch.distributed.run, one rank per GPU)
# ---------------------------------------------------------------------------------------------
def bench_main(args, metric, query, cpu_baseline_fn=None, roofline_fn=None, traffic_fn=None):
    import sys

    import torch
    import torch.distributed as dist

    from . import lib
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # QE_DIST_BACKEND=gloo rehearses the multi-rank path on fewer GPUs than ranks (host-staged
    # exchange); production is nccl = RCCL, one rank per GPU
    backend = os.environ.get("QE_DIST_BACKEND", "nccl")
    dev = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(dev)
    solo = world == 1                  # the plan alone on one GPU (bench.py --plan dist): no group
    if not solo and not dist.is_initialized():
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{dev}"))
        else:
            dist.init_process_group(backend)
    ctx = lib.Ctx(dev)
    eng = GPUEngine(ctx, rank, world)
    total_rows = args.rows * world                 # weak scaling: every rank owns args.rows per relation
    kinds = [("mod", total_rows), ("mod", total_rows), ("hi32",)]
    for r in range(4):
        ctx.gen_relation(total_rows, kinds, seed=args.seed, gen_rel=r)
    ctx.sync()
    ex = DistExecutor(eng, [total_rows] * 4)
    out = None
    for _ in range(args.warmup):
        out, rows = ex.run(query)
    ctx.set_profiling(True)
    ctx.reset_stats()
    if not solo:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out, rows = ex.run(query)
    ctx.sync()
    torch.cuda.synchronize()
    if not solo:
        dist.barrier()
    dt = time.perf_counter() - t0
    if not solo:
        tmax = torch.tensor([dt], dtype=torch.float64, device=f"cuda:{dev}" if backend == "nccl" else "cpu")
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        dt = float(tmax.item())
    stats = ctx.kernel_stats()
    ctx.set_profiling(False)
    res = None
    if rank == 0:
        kern = sorted(stats.items(), key=lambda kv: -kv[1]["ms"])
        res = {
            "metric": metric, "value": round(rows * args.steps / dt, 1), "unit": "joined tuples/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "u64",
            "data": "synthetic: splitmix64 relations generated in HBM (SURVEY.md §9.1), seed %d" % args.seed,
            "config": {"workload": "C3: 4-relation chain join, 2 filters on R3, %d rows/rel per GPU "
                                   "(%d rows/rel in total)" % (args.rows, total_rows),
                       "query": query.strip(), "rows_per_relation": total_rows, "result_rows": rows,
                       "stdout": out, "executor": "qe.dist key-partitioned plan, RCCL all-to-all per join",
                       "parallelism": f"hash-partitioned dp{world}"},
            "roofline": roofline_fn(stats, traffic_fn() if traffic_fn else None) if roofline_fn else None,
            "stages": {k: {"ms_per_step": round(s["ms"] / args.steps, 3)} for k, s in kern[:10]},
            "cpu_baseline": None,
        }
    if not solo:
        dist.barrier()
    ctx.close()
    if not solo:
        dist.destroy_process_group()
    if rank == 0:
        print(f"[bench] rank 0 done: {out.strip()!r}", file=sys.stderr)
    return res
