"""Key-partitioned multi-GPU execution of join queries.

One process per GPU (torch.distributed; backend "nccl" = RCCL over xGMI).  Every rank holds a
replica of the base columns and owns a contiguous rowid slice of every relation.  A query runs
as a relational plan over the device primitives of libqe:

  filters   -- each rank scans its own slice (qe_filter_scan_range); a second filter on the same
               binding refines it and prints the global count (all-reduce), as the reference's
               exec_filter_rel_exists does (src/filter.c:3-35)
  joins     -- both inputs are gathered to keys (replicated columns, local), hash-partitioned on
               the key (qe_partition: dest = fmix64(key) % world), exchanged with one RCCL
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

    __slots__ = ("ptr", "n", "keep", "free")

    def __init__(self, ptr, n, keep=None, free=None):
        self.ptr, self.n, self.keep, self.free = ptr, n, keep, free

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
        return DArr(p.key, p.n, keep=p, free=lambda: ctx.pairs_free(p))

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
        outs = []
        for src, dt in [(sk, torch.int64)] + [(t, torch.int32) for t in sc]:
            s = src[:n].to(self.comm_dev) if self.comm_dev != dev else src[:n]
            r = torch.empty(max(1, total), dtype=dt, device=self.comm_dev)
            dist.all_to_all_single(r[:total], s, out_splits, counts, group=self.group)
            if self.comm_dev != dev:
                r = r.to(dev)
            outs.append(r)
        torch.cuda.synchronize()
        rk = DArr(outs[0].data_ptr(), total, keep=outs[0])
        rc = [DArr(t.data_ptr(), total, keep=t) for t in outs[1:]]
        return rk, rc


# ---------------------------------------------------------------------------------------------
# the plan
# ---------------------------------------------------------------------------------------------
class DistExecutor:
    """Runs one query line with the key-partitioned relational plan on `engine`."""

    def __init__(self, engine, rel_rows: list[int]):
        self.e = engine
        self.rel_rows = rel_rows

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
        comp_of: dict[int, int] = {}          # binding -> component id
        comps: dict[int, dict[int, DArr]] = {}  # component -> {binding: rowids}
        lists: dict[int, DArr] = {}           # filtered, not yet joined bindings

        def need_after(k):
            need = {b for (b, _) in sels}
            for p in preds[k + 1:]:
                need.add(p.a[0])
                if p.b:
                    need.add(p.b[0])
            return need

        def component(b):
            if b in comp_of:
                return comp_of[b]
            cid = len(comps) + 1000 * (b + 1)
            comps[cid] = {b: lists.pop(b) if b in lists else self._base(rels[b])}
            comp_of[b] = cid
            return cid

        for k, p in enumerate(preds):
            if p.kind == "filter":
                b, c = p.a
                rel = rels[b]
                if b in comp_of:
                    cid = comp_of[b]
                    idx = e.filter_idx(rel, c, comps[cid][b], p.op, p.const)
                    comps[cid] = {bb: e.take(r, idx) for bb, r in comps[cid].items()}
                    out.append(f"{e.allreduce(e.length(comps[cid][b])) & 0xFFFFFFFF:d}\n")
                elif b in lists:
                    lists[b] = e.refine(rel, c, lists[b], p.op, p.const)
                    out.append(f"{e.allreduce(e.length(lists[b])):d}\n")
                else:
                    s, t = owned_range(self.rel_rows[rel], e.rank, e.world)
                    lists[b] = e.scan(rel, c, s, t, p.op, p.const)
                continue
            (ba, ca), (bb, cb) = p.a, p.b
            A, B = component(ba), component(bb)
            need = need_after(k)
            if A == B:
                cols = comps[A]
                idx = e.keep_equal(e.keys(rels[ba], ca, cols[ba]), e.keys(rels[bb], cb, cols[bb]))
                comps[A] = {x: e.take(r, idx) for x, r in cols.items()}
                continue
            ka = e.keys(rels[ba], ca, comps[A][ba])
            kb = e.keys(rels[bb], cb, comps[B][bb])
            sides = []
            for cid, kk in ((A, ka), (B, kb)):
                cols = comps[cid]
                keep = [x for x in sorted(cols) if x in need] or [sorted(cols)[0]]
                if e.world > 1:
                    if len(keep) > 4:
                        raise NotSupported("more than 4 rowid columns in one exchange")
                    rk, rc = e.exchange(kk, [cols[x] for x in keep])
                    sides.append((rk, dict(zip(keep, rc))))
                else:
                    sides.append((kk, {x: cols[x] for x in keep}))
            (rka, ca_cols), (rkb, cb_cols) = sides
            ia, ib = e.join_local(rka, rkb)
            merged = {x: e.take(r, ia) for x, r in ca_cols.items()}
            merged.update({x: e.take(r, ib) for x, r in cb_cols.items()})
            del comps[A], comps[B]
            comps[A] = merged
            for x in list(comp_of):
                if comp_of[x] in (A, B):
                    comp_of[x] = A
            for x in merged:
                comp_of[x] = A
        # print_sums
        roots = {comp_of[b] for (b, _) in sels}
        if len(roots) != 1:
            raise NotSupported("disconnected selects")
        cid = roots.pop()
        anyb = next(iter(comps[cid]))
        rows = e.allreduce(e.length(comps[cid][anyb]))
        line_out = []
        for (b, c) in sels:
            s = e.allreduce(e.checksum(rels[b], c, comps[cid][b]))
            line_out.append("NULL " if rows == 0 else f"{s} ")
        out.append("".join(line_out) + "\n")
        return "".join(out), rows


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
    if not dist.is_initialized():
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
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out, rows = ex.run(query)
    ctx.sync()
    torch.cuda.synchronize()
    dist.barrier()
    dt = time.perf_counter() - t0
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
    dist.barrier()
    ctx.close()
    dist.destroy_process_group()
    if rank == 0:
        print(f"[bench] rank 0 done: {out.strip()!r}", file=sys.stderr)
    return res
