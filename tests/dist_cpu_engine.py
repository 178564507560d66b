"""A numpy engine for qe.dist.DistAggJoin (the C5 skew plan) so it runs under torch.distributed
gloo on CPU.  TEST INFRASTRUCTURE ONLY: the product engine is qe.dist.GPUEngine (libqe).  (The
relational plan is C: tests/plan_engine.py drives it.)"""
import os
import socket

import numpy as np

from qe.dist import M64

_OPS = {"=": np.equal, ">": np.greater, "<": np.less}


def part_of(k: np.ndarray, nparts: int) -> np.ndarray:
    """qe_partition's destination: (hi32((k ^ k >> 29) * 0xbf58476d1ce4e5b9) * nparts) >> 32"""
    k = np.asarray(k, dtype=np.uint64)
    with np.errstate(over="ignore"):
        h = (k ^ (k >> np.uint64(29))) * np.uint64(0xbf58476d1ce4e5b9)
    return ((h >> np.uint64(32)) * np.uint64(nparts)) >> np.uint64(32)


class NumpyEngine:
    def __init__(self, rels, rank, world, group=None):
        self.rels, self.rank, self.world, self.group = rels, rank, world, group
        self.exchanges = 0

    def base_side_light(self, rel, col, heavy):
        c = self.rels[rel][col]
        mask = part_of(c, self.world) == np.uint64(self.rank)
        mask &= ~np.isin(c, np.asarray(heavy, dtype=np.uint64))
        rows = np.nonzero(mask)[0].astype(np.uint32)
        return c[rows], rows

    def join_count_sums(self, ka, va, kb, vb, sel_a, sel_b):
        ua, ca = np.unique(ka, return_counts=True)
        ub, cb = np.unique(kb, return_counts=True)
        wa = np.zeros(len(ka), np.uint64)        # partners of each A row
        pos = np.searchsorted(ub, ka)
        hit = (pos < len(ub)) & (ub[np.minimum(pos, len(ub) - 1)] == ka)
        wa[hit] = cb[pos[hit]]
        wb = np.zeros(len(kb), np.uint64)
        pos = np.searchsorted(ua, kb)
        hit = (pos < len(ua)) & (ua[np.minimum(pos, len(ua) - 1)] == kb)
        wb[hit] = ca[pos[hit]]
        ra = va if va is not None else np.arange(len(ka))
        rb = vb if vb is not None else np.arange(len(kb))
        with np.errstate(over="ignore"):
            sa = [int(np.sum(self.rels[r][c][ra] * wa, dtype=np.uint64)) for (r, c) in sel_a]
            sb = [int(np.sum(self.rels[r][c][rb] * wb, dtype=np.uint64)) for (r, c) in sel_b]
        return int(np.sum(wa, dtype=np.uint64)), sa, sb

    def heavy_stats(self, rel, col, start, end, heavy, val=None, weights=None):
        k = self.rels[rel][col][start:end]
        heavy = np.asarray(heavy, dtype=np.uint64)
        counts = np.array([np.sum(k == h) for h in heavy], dtype=np.uint64)
        if weights is None:
            return counts, None
        v = self.rels[val[0]][val[1]][start:end]
        s = 0
        for h, w in zip(heavy.tolist(), np.asarray(weights).tolist()):
            s = (s + int(np.sum(v[k == h], dtype=np.uint64)) * int(w)) & M64
        return counts, s

    def column_prefix(self, rel, col, m):
        return self.rels[rel][col][:m]

    def allreduce_vec(self, a):
        a = np.ascontiguousarray(a, dtype=np.uint64)
        if self.world == 1 or a.size == 0:
            return a
        import torch
        import torch.distributed as dist
        t = torch.from_numpy(a.view(np.int64).copy())
        dist.all_reduce(t, group=self.group)
        return t.numpy().view(np.uint64)


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def agg_worker(rank, world, port, rels, queries, outq, sample):
    """one gloo rank of the aggregate (skew) plan"""
    import torch.distributed as dist
    from qe.dist import DistAggJoin
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        eng = NumpyEngine(rels, rank, world)
        ex = DistAggJoin(eng, [len(r[0]) for r in rels], sample=sample)
        res = [ex.run(q) for q in queries]
        if rank == 0:
            outq.put((res, 0))
    finally:
        dist.destroy_process_group()
