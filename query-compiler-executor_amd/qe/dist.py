"""The skewed 2-relation join across ranks in aggregate form (C5, SURVEY.md §8(e) "Skew").

The relational join plan for N ranks is host C (include/qe_plan.h, host/qe_plan.c), driven
through libqe's qe_run_queries_dist over an RCCL communicator.  What stays here is the C5 leg: a
single equi-join too large to materialise (3.8e14 pairs at 1e9 rows/side), computed as
sum_k (sum_{r in R_k} col(r)) * |S_k| with the Zipf head split across ranks -- driven from
Python over torch.distributed (backend "nccl" = RCCL) and libqe's primitives.

The executor is engine-agnostic: GPUEngine drives libqe; tests/dist_cpu_engine.py supplies a numpy
engine to run the same plan under gloo on CPU.
"""
from __future__ import annotations

import os
import re

import numpy as np

M64 = (1 << 64) - 1


class NotSupported(Exception):
    pass


def parse(line: str):
    """`rels|preds|selects` of a well-formed line (src/parsing.c's grammar): ([rel], [("join", (b, c),
    (b, c)) | ("filter", ...)], [(b, c)]) -- the aggregate plan needs the one join and the selects"""
    rels_s, preds_s, sel_s = line.strip().split("|")
    rels = [int(x) for x in rels_s.split(" ")]
    preds = []
    for p in preds_s.split("&"):
        m = re.fullmatch(r"(\d+)\.(\d+)(.)(\d+)\.(\d+)", p)
        if m:
            a, b, _, c, d = m.groups()
            preds.append(("join", (int(a), int(b)), (int(c), int(d))))
        else:
            preds.append(("filter", p, None))
    sels = [tuple(int(v) for v in s.split(".")) for s in sel_s.split(" ")]
    return rels, preds, sels


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

    def base_side_light(self, rel, col, heavy):
        """base_side without the heavy keys (skew path): the local bucket minus heavy keys"""
        if self.world == 1 and len(heavy) == 0:          # one rank: the column itself (zero copy)
            c = self.ctx.column(rel, col)
            return DArr(c.d, c.n, bits=self.ctx.column_bits(rel, col)), None
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
        joins = [p for p in preds if p[0] == "join"]
        if len(rels) != 2 or len(preds) != 1 or len(joins) != 1 or joins[0][1][0] == joins[0][2][0]:
            raise NotSupported("aggregate plan: exactly one join between two bindings, no filters")
        (ba, ca), (bb, cb) = joins[0][1], joins[0][2]
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
