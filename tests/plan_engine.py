"""A numpy (+ torch.distributed gloo) engine for the C partitioned plan (include/qe_plan.h) through
ctypes, so the plan that drives libqe + RCCL on the GPUs -- the same compiled C -- runs on CPU
ranks here.  TEST INFRASTRUCTURE ONLY: the product engine is libqe's (qe_run_queries_dist)."""
from __future__ import annotations

import ctypes as C
import os
import traceback

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO = os.path.join(ROOT, "query-compiler-executor_amd", "build", "libqeplan.so")

_OPS = {"=": np.equal, ">": np.greater, "<": np.less}
I, U32, U64, VP, H = C.c_int, C.c_uint32, C.c_uint64, C.c_void_p, C.c_uint64
P = C.POINTER

FIELDS = [
    ("rel_count", C.CFUNCTYPE(I, VP, P(U32))),
    ("rel_shape", C.CFUNCTYPE(I, VP, U32, P(U64), P(U32))),
    ("scan", C.CFUNCTYPE(I, VP, U32, U32, U64, U64, C.c_char, U64, P(H))),
    ("iota", C.CFUNCTYPE(I, VP, U64, U64, P(H))),
    ("refine", C.CFUNCTYPE(I, VP, U32, U32, H, C.c_char, U64, P(H))),
    ("keys", C.CFUNCTYPE(I, VP, U32, U32, H, P(H))),
    ("base_side", C.CFUNCTYPE(I, VP, U32, U32, P(H), P(H))),
    ("exchange_start", C.CFUNCTYPE(I, VP, H, P(H), I, P(H))),
    ("exchange_finish", C.CFUNCTYPE(I, VP, H, P(H), P(H))),
    ("join", C.CFUNCTYPE(I, VP, H, H, H, H, P(H), P(H))),
    ("take", C.CFUNCTYPE(I, VP, H, H, P(H))),
    ("length", C.CFUNCTYPE(I, VP, H, P(U64))),
    ("checksums", C.CFUNCTYPE(I, VP, I, P(U32), P(U32), P(H), P(U64))),
    ("allreduce", C.CFUNCTYPE(I, VP, P(U64), I)),
    ("release", C.CFUNCTYPE(None, VP, H)),
    ("fallback", C.CFUNCTYPE(I, VP, VP, VP)),
    ("scan2", C.CFUNCTYPE(I, VP, U32, U32, C.c_char, U64, U32, C.c_char, U64, U64, U64, I, P(H))),
    ("join_carry", C.CFUNCTYPE(I, VP, H, H, H, H, I, P(H), H, P(H), P(H), P(H), P(H))),
    ("join_sums", C.CFUNCTYPE(I, VP, H, H, H, H, I, P(H), I, P(I), P(U32), P(U32), P(U64), P(U64))),
    ("values", C.CFUNCTYPE(I, VP, U32, U32, H, P(H))),
]
VALUES, VALUES_SRC = 0xFFFFFFFF, 4   # include/qe_plan.h: QE_PLAN_VALUES, QE_PLAN_VALUES_SRC


JOIN_AGG = C.CFUNCTYPE(I, VP, U32, U32, U32, U32, I, P(I), P(U32), P(U64), P(U64))
COLUMN = C.CFUNCTYPE(I, VP, U32, U32, P(H))
KEYS_OF = C.CFUNCTYPE(I, VP, U32, U32, H, P(H))
BASE_SIDE_ALL = C.CFUNCTYPE(I, VP, U32, U32, P(H), P(H))


class Engine(C.Structure):
    _fields_ = [("u", VP), ("rank", U32), ("world", U32)] + FIELDS + [("mat_limit", P(U64)), ("join_agg", JOIN_AGG),
                                                                      ("column", COLUMN), ("keys_of", KEYS_OF),
                                                                      ("base_side_all", BASE_SIDE_ALL)]


def part_of(k: np.ndarray, nparts: int) -> np.ndarray:
    """qe_partition's destination: (hi32((k ^ k >> 29) * 0xbf58476d1ce4e5b9) * nparts) >> 32"""
    k = np.asarray(k, dtype=np.uint64)
    with np.errstate(over="ignore"):
        h = (k ^ (k >> np.uint64(29))) * np.uint64(0xbf58476d1ce4e5b9)
    return ((h >> np.uint64(32)) * np.uint64(nparts)) >> np.uint64(32)


def join_local(ka, kb):
    """every (i, j) with ka[i] == kb[j]: i ascending by key (stable), j in kb's stable key order"""
    oa = np.argsort(ka, kind="stable")
    ob = np.argsort(kb, kind="stable")
    sa, sb = ka[oa], kb[ob]
    lo = np.searchsorted(sb, sa, "left")
    hi = np.searchsorted(sb, sa, "right")
    c = hi - lo
    ia = np.repeat(oa, c)
    starts = np.repeat(lo - np.concatenate([[0], np.cumsum(c)[:-1]]).astype(np.int64), c)
    ib = ob[starts + np.arange(int(c.sum()))]
    return ia.astype(np.uint32), ib.astype(np.uint32)


class NumpyPlanEngine:
    """one rank: relations replicated as numpy columns; handles index a dict of arrays"""

    def __init__(self, rels, rank=0, world=1, group=None, fused_scan=True, join_carry=True, join_sums=True, values=True,
                 join_agg=True, key_carry=True):
        self.rels, self.rank, self.world, self.group = rels, rank, world, group
        self.h, self.next, self.borrowed = {}, 1, set()
        self.exchanges = 0
        self.sums_calls = 0                      # last joins run in aggregate form (join_sums)
        self.values_calls = 0                    # bindings whose select values ride instead of rowids
        self.scan2_values = 0                    # fused scans asked to emit their col1 values
        self.mat_limit = 1 << 62
        self.lib = C.CDLL(SO)
        self.lib.qe_plan_run_text.argtypes = [P(Engine), C.c_char_p, P(C.c_void_p), P(C.c_size_t), P(U64), P(U64)]
        self.lib.qe_plan_check_text.argtypes = [P(Engine), C.c_char_p, P(C.c_uint8), C.c_size_t]
        self.lib.qe_plan_why.restype = C.c_char_p
        self.libc = C.CDLL(None)
        self.libc.free.argtypes = [C.c_void_p]
        self._cbs = []
        e = Engine()
        e.u, e.rank, e.world = None, rank, world
        for name, ftype in FIELDS:
            if (name == "fallback" or (name == "scan2" and not fused_scan) or (name == "join_carry" and not join_carry)
                    or (name == "join_sums" and not join_sums) or (name == "values" and not values)):
                setattr(e, name, ftype())            # NULL: refused queries return QE_ENOTSUP; no fused scan
                continue
            fn = self._wrap(getattr(self, "cb_" + name), name == "release")
            cb = ftype(fn)
            self._cbs.append(cb)
            setattr(e, name, cb)
        if join_agg:
            self._agg_cb = JOIN_AGG(self._wrap(self.cb_join_agg, False))
            e.join_agg = self._agg_cb
        self.agg_calls = 0                       # last joins of two base relations in aggregate form
        self.keys_of_calls = 0                   # join keys that rode with their rows (no gather)
        self.values_rows = 0                     # base sides whose rows rode as a column's values
        self.bcast_sides = 0                     # whole base sides taken by broadcast joins
        self._bsa_cb = BASE_SIDE_ALL(self._wrap(self.cb_base_side_all, False))
        e.base_side_all = self._bsa_cb
        if key_carry:
            self._col_cb = COLUMN(self._wrap(self.cb_column, False))
            self._ko_cb = KEYS_OF(self._wrap(self.cb_keys_of, False))
            e.column, e.keys_of = self._col_cb, self._ko_cb
        self.e = e
        self._limit = None

    def set_global_limit(self, pairs):
        """the plan's own check of a join's all-ranks pair count (qe_engine.mat_limit); None: off"""
        self._limit = None if pairs is None else U64(pairs)
        self.e.mat_limit = C.pointer(self._limit) if pairs is not None else P(U64)()

    # -- plumbing
    def _wrap(self, f, void):
        def g(*a):
            try:
                r = f(*a)
                return None if void else (0 if r is None else r)
            except Exception:
                traceback.print_exc()
                return None if void else -1
        return g

    def put(self, arr, borrowed=False) -> int:
        k = self.next
        self.next += 1
        self.h[k] = arr
        if borrowed:
            self.borrowed.add(k)
        return k

    def get(self, k):
        return self.h[k]

    # -- the C entry points
    def run(self, text: str):
        """(stdout, rc, rows, refused)"""
        out, n, rows, nref = C.c_void_p(), C.c_size_t(), U64(), U64()
        rc = self.lib.qe_plan_run_text(C.byref(self.e), text.encode(), C.byref(out), C.byref(n), C.byref(rows),
                                       C.byref(nref))
        s = C.string_at(out, n.value).decode("latin-1") if out.value else ""
        if out.value:
            self.libc.free(out)
        return s, rc, rows.value, nref.value

    def check(self, text: str):
        acc = (C.c_uint8 * 4096)()
        nq = self.lib.qe_plan_check_text(C.byref(self.e), text.encode(), acc, 4096)
        return [bool(acc[i]) for i in range(nq)], self.lib.qe_plan_why().decode()

    def live_handles(self) -> int:
        return len(self.h) - len(self.borrowed)

    # -- engine callbacks
    def cb_rel_count(self, u, n):
        n[0] = len(self.rels)

    def cb_rel_shape(self, u, rel, rows, ncols):
        if rel >= len(self.rels):
            return -1
        rows[0] = len(self.rels[rel][0]) if self.rels[rel] else 0
        ncols[0] = len(self.rels[rel])

    def _unordered(self, rows):
        """like libqe's unordered scans: the plan must not depend on a list's order"""
        return np.random.default_rng(len(rows) + 31 * self.rank).permutation(rows).astype(np.uint32)

    def cb_scan(self, u, rel, col, s, t, op, v, out):
        c = self.rels[rel][col][s:t]
        out[0] = self.put(self._unordered(np.nonzero(_OPS[op.decode()](c, np.uint64(v)))[0] + s))

    def cb_scan2(self, u, rel, c1, op1, v1, c2, op2, v2, s, t, values, out):
        self.scan2_values += bool(values & 1)      # (bits 8..15: a join-key hint this engine ignores)
        a = self.rels[rel][c1][s:t]
        b = self.rels[rel][c2][s:t]
        m = _OPS[op1.decode()](a, np.uint64(v1)) & _OPS[op2.decode()](b, np.uint64(v2))
        out[0] = self.put(self._unordered(np.nonzero(m)[0] + s))

    def cb_iota(self, u, s, n, out):
        out[0] = self.put(np.arange(s, s + n, dtype=np.uint32))

    def cb_refine(self, u, rel, col, rows, op, v, out):
        r = self.h.pop(rows)
        out[0] = self.put(r[_OPS[op.decode()](self.rels[rel][col][r], np.uint64(v))])

    def cb_keys(self, u, rel, col, rows, out):
        out[0] = self.put(self.rels[rel][col][self.get(rows)])

    def cb_base_side(self, u, rel, col, keys, rowids):
        c = self.rels[rel][col]
        if self.world == 1:
            keys[0] = self.put(c, borrowed=True)
            rowids[0] = 0
            return
        mask = part_of(c, self.world) == np.uint64(self.rank)
        rows = np.nonzero(mask)[0]
        # an unordered bucket, like qe_bucket_select's: shuffle so no test depends on its order
        rows = np.random.default_rng(self.rank + 17).permutation(rows).astype(np.uint32)
        keys[0] = self.put(c[rows])
        rowids[0] = self.put(rows)

    def cb_base_side_all(self, u, rel, col, keys, rowids):
        """the whole column at any rank count (the plan's broadcast joins), as at one rank"""
        self.bcast_sides += 1
        keys[0] = self.put(self.rels[rel][col], borrowed=True)
        rowids[0] = 0

    def cb_exchange_start(self, u, keys, cols, ncols, ticket):
        import torch
        import torch.distributed as dist
        self.exchanges += 1
        k = self.h.pop(keys)
        cs = [self.h.pop(cols[i]) for i in range(ncols)]
        dest = part_of(k, self.world).astype(np.int64)
        order = np.argsort(dest, kind="stable")
        counts = np.bincount(dest, minlength=self.world).astype(np.int64)
        cnt = torch.from_numpy(counts)
        rcnt = torch.empty_like(cnt)
        dist.all_to_all_single(rcnt, cnt, group=self.group)
        osp, isp = rcnt.tolist(), counts.tolist()
        outs = []
        for arr, dt in [(k.view(np.int64), torch.int64)] + [(c.view(np.int32), torch.int32) for c in cs]:
            s = torch.from_numpy(np.ascontiguousarray(arr[order]))
            r = torch.empty(sum(osp), dtype=dt)
            dist.all_to_all_single(r, s, osp, isp, group=self.group)
            outs.append(r.numpy())
        ticket[0] = self.put((outs[0].view(np.uint64), [o.view(np.uint32) for o in outs[1:]]))

    def cb_exchange_finish(self, u, ticket, keys, cols):
        k, cs = self.h.pop(ticket)
        keys[0] = self.put(k)
        for i, c in enumerate(cs):
            cols[i] = self.put(c)

    def cb_join(self, u, ka, va, kb, vb, oa, ob):
        ia, ib = join_local(self.get(ka), self.get(kb))
        if len(ia) > self.mat_limit:          # like qe_join_pairs: QE_ETOOBIG past the limit
            return -5
        oa[0] = self.put(self.get(va)[ia] if va else ia)
        ob[0] = self.put(self.get(vb)[ib] if vb else ib)

    def cb_join_carry(self, u, ka, va, kb, vb, nb, cb, xa, oa, ob, outb, outxa):
        ia, ib = join_local(self.get(ka), self.get(kb))
        if len(ia) > self.mat_limit:
            return -5
        vals = self.get(va) if va else None
        if isinstance(vals, tuple):              # a whole column whose binding rides as another column's values
            assert vals[0] == "column" and len(vals[1]) == len(self.get(ka))
            ra = ia
            oa[0] = self.put(vals[1][ia].astype(np.uint32))
            self.values_rows += 1
        else:
            ra = vals[ia] if va else ia          # a's rowids (a whole column: positions are rowids)
            oa[0] = self.put(ra)
        ob[0] = self.put(self.get(vb)[ib] if vb else ib)
        for k in range(nb):
            outb[k] = self.put(self.get(cb[k])[ib])
        if xa:
            tag, col = self.get(xa)
            assert tag == "column"
            outxa[0] = self.put(col[ra].astype(np.uint32))

    def cb_column(self, u, rel, col, out):
        c = self.rels[rel][col]
        if len(c) and int(c.max()) >> 32:
            return -6                            # QE_ENOTSUP: the key is gathered later
        out[0] = self.put(("column", c))

    def cb_keys_of(self, u, rel, col, vals, out):
        self.keys_of_calls += 1
        out[0] = self.put(self.get(vals).astype(np.uint64))

    def cb_join_sums(self, u, ka, va, kb, vb, nb, cb, nsel, src, rels, cols, pairs, sums):
        """aggregate form, computed independently of the join: each b row counts its a partners"""
        self.sums_calls += 1
        a, b = self.get(ka), self.get(kb)
        sa = np.sort(a, kind="stable")
        cnt = (np.searchsorted(sa, b, "right") - np.searchsorted(sa, b, "left")).astype(np.uint64)
        total = int(cnt.sum())
        if total > self.mat_limit:
            return -5
        pairs[0] = total
        for s in range(nsel):
            k = src[s] & 3
            rows = (self.get(vb) if vb else np.arange(len(b), dtype=np.uint32)) if k == 0 else self.get(cb[k - 1])
            vals = rows.astype(np.uint64) if src[s] & VALUES_SRC else self.rels[rels[s]][cols[s]][rows]
            with np.errstate(over="ignore"):
                sums[s] = int(np.sum(cnt * vals, dtype=np.uint64))

    def cb_join_agg(self, u, ra, ca, rb, cb, nsel, side, cols, pairs, sums):
        """this rank's share: its row slice of each side, each row weighted by its key's partner
        count in the other (replicated) side -- the shares add up to the join's numbers"""
        self.agg_calls += 1
        ka, kb = self.rels[ra][ca], self.rels[rb][cb]
        sa, sb = np.sort(ka), np.sort(kb)
        def slice_of(n):
            return n * self.rank // self.world, n * (self.rank + 1) // self.world
        a0, a1 = slice_of(len(ka))
        b0, b1 = slice_of(len(kb))
        ca_ = (np.searchsorted(sb, ka[a0:a1], "right") - np.searchsorted(sb, ka[a0:a1], "left")).astype(np.uint64)
        cb_ = (np.searchsorted(sa, kb[b0:b1], "right") - np.searchsorted(sa, kb[b0:b1], "left")).astype(np.uint64)
        pairs[0] = int(ca_.sum())
        with np.errstate(over="ignore"):
            for s in range(nsel):
                if side[s] == 0:
                    sums[s] = int(np.sum(ca_ * self.rels[ra][cols[s]][a0:a1], dtype=np.uint64))
                else:
                    sums[s] = int(np.sum(cb_ * self.rels[rb][cols[s]][b0:b1], dtype=np.uint64))

    def cb_values(self, u, rel, col, rows, out):
        c = self.rels[rel][col]
        if len(c) and int(c.max()) >> 32:
            return -6                            # QE_ENOTSUP: the rowids stay
        self.values_calls += 1
        out[0] = self.put(c[self.get(rows)].astype(np.uint32))

    def cb_take(self, u, src, idx, out):
        out[0] = self.put(self.get(src)[self.get(idx)])

    def cb_length(self, u, h, n):
        n[0] = len(self.get(h))

    def cb_checksums(self, u, n, rels, cols, rows, sums):
        for i in range(n):
            r = self.get(rows[i])
            v = r.astype(np.uint64) if rels[i] == VALUES else self.rels[rels[i]][cols[i]][r]
            sums[i] = int(np.sum(v, dtype=np.uint64))

    def cb_allreduce(self, u, v, n):
        if self.world == 1 or n == 0:
            return
        import torch
        import torch.distributed as dist
        a = np.array([v[i] for i in range(n)], dtype=np.uint64)
        t = torch.from_numpy(a.view(np.int64).copy())
        dist.all_reduce(t, group=self.group)
        r = t.numpy().view(np.uint64)
        for i in range(n):
            v[i] = int(r[i])

    def cb_release(self, u, h):
        if h in self.borrowed:
            return
        self.h.pop(h, None)


def free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def worker(rank, world, port, rels, queries, outq, limits=None, global_limit=None, opts=None):
    """one gloo rank: every query through the C plan, rank 0 reports (stdout, rc, rows, refused);
    limits[rank] (optional): that rank's materialisation limit (its local joins); global_limit
    (optional): the plan's limit on a join's all-ranks pair count"""
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    opts = dict(opts or {})
    for k, v in (opts.pop("env", None) or {}).get(rank, {}).items():   # this rank's own environment
        os.environ[k] = v
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        eng = NumpyPlanEngine(rels, rank, world, **opts)
        if limits:
            eng.mat_limit = limits[rank]
        if global_limit is not None:
            eng.set_global_limit(global_limit)
        res = [eng.run(q) for q in queries]
        if rank == 0:
            outq.put((res, eng.exchanges, eng.live_handles()))
    finally:
        dist.destroy_process_group()
