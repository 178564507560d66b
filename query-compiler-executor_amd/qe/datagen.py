"""Synthetic relations for the join path.

Counter-based splitmix64: ``v(seed, rel, col, row) = splitmix64(((seed<<40)|(rel<<36)|(col<<32)) + row)``.
Column kinds:

* ``("mod", M)``  -> ``v % M``       (join keys; SURVEY uses M = N)
* ``("hi32",)``   -> ``v >> 32``     (filter / payload column, uniform in [0, 2^32))
* ``("zipf", D, theta, perm_seed)``  -> Zipf(theta) rank over [0, D) mapped through a shared
  rank->key permutation (config 5 shape): rank = #{r : cdf[r] <= u} for the 53-bit uniform u of
  v, capped at D-1, then key = feistel_perm(rank) -- a seeded 4-round Feistel bijection of
  [0, 2^b) cycle-walked into [0, D).  Given the same CDF table, libqe's device sampler
  (qe_set_zipf_table + kind 2) draws the same keys bit for bit.

The same generator runs on the GPU inside libqe (``qe_gen_column``); tests check the two agree
bit for bit.  Files use the reference's binary layout: ``u64 rows, u64 ncols`` then the columns
column-major (reference src/utilities.c:105-121).
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field

import numpy as np

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)
GOLDEN_GAMMA = np.uint64(0x9E3779B97F4A7C15)
MUL1 = np.uint64(0xBF58476D1CE4E5B9)
MUL2 = np.uint64(0x94D049BB133111EB)


def splitmix64(x: np.ndarray) -> np.ndarray:
    """Vectorised splitmix64 finaliser on uint64 (wrapping arithmetic)."""
    with np.errstate(over="ignore"):
        z = x.astype(np.uint64) + GOLDEN_GAMMA
        z = (z ^ (z >> np.uint64(30))) * MUL1
        z = (z ^ (z >> np.uint64(27))) * MUL2
        return z ^ (z >> np.uint64(31))


def splitmix64_int(x: int) -> int:
    m = (1 << 64) - 1
    z = (x + 0x9E3779B97F4A7C15) & m
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & m
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & m
    return z ^ (z >> 31)


def stream_base(seed: int, rel: int, col: int) -> int:
    return ((seed << 40) | (rel << 36) | (col << 32)) & ((1 << 64) - 1)


def raw_column(seed: int, rel: int, col: int, rows: int, start: int = 0) -> np.ndarray:
    base = np.uint64(stream_base(seed, rel, col))
    idx = np.arange(start, start + rows, dtype=np.uint64)
    with np.errstate(over="ignore"):
        return splitmix64(idx + base)


def zipf_cdf(domain: int, theta: float) -> np.ndarray:
    """Cumulative Zipf(theta) weights over ranks 1..domain, normalised to [0, 1]."""
    w = 1.0 / np.power(np.arange(1, domain + 1, dtype=np.float64), theta)
    c = np.cumsum(w)
    return c / c[-1]


def feistel_perm(x: np.ndarray, domain: int, perm_seed: int) -> np.ndarray:
    """Seeded bijection of [0, domain): 4 Feistel rounds (round function splitmix64) on b-bit
    words, b = bit length of domain-1 rounded up to even (>= 2), cycle-walked until < domain."""
    b = max(2, int(domain - 1).bit_length())
    b += b & 1
    h = np.uint64(b // 2)
    mask = np.uint64((1 << (b // 2)) - 1)
    keys = [np.uint64(stream_base(perm_seed, 15, r)) for r in range(4)]
    x = np.asarray(x, dtype=np.uint64).copy()
    todo = np.arange(len(x))
    dom = np.uint64(domain)
    first = True
    while first or len(todo):
        first = False
        y = x[todo]
        lo, hi = y & mask, y >> h
        with np.errstate(over="ignore"):
            for k in keys:
                lo, hi = hi ^ (splitmix64(lo + k) & mask), lo
        y = (hi << h) | lo
        x[todo] = y
        todo = todo[y >= dom]
    return x


def zipf_perm(domain: int, perm_seed: int) -> np.ndarray:
    """Rank -> key permutation shared by both sides of a skewed join (seeded)."""
    return feistel_perm(np.arange(domain, dtype=np.uint64), domain, perm_seed)


def zipf_ranks(v: np.ndarray, cdf: np.ndarray) -> np.ndarray:
    u = (v >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)   # 53-bit uniform
    rank = np.searchsorted(cdf, u, side="right")
    return np.minimum(rank, len(cdf) - 1).astype(np.uint64)


def column(seed: int, rel: int, col: int, rows: int, kind: tuple, start: int = 0) -> np.ndarray:
    v = raw_column(seed, rel, col, rows, start)
    if kind[0] == "mod":
        return v % np.uint64(kind[1])
    if kind[0] == "hi32":
        return v >> np.uint64(32)
    if kind[0] == "zipf":
        domain, theta, perm_seed = int(kind[1]), float(kind[2]), int(kind[3])
        return feistel_perm(zipf_ranks(v, zipf_cdf(domain, theta)), domain, perm_seed)
    raise ValueError(f"unknown column kind {kind!r}")


@dataclass
class RelSpec:
    rows: int
    kinds: list = field(default_factory=list)   # one kind tuple per column


def chain_spec(n_rels: int, rows: int, key_domain: int | None = None) -> list[RelSpec]:
    """every relation has c0 = v % N, c1 = v % N, c2 = v >> 32."""
    d = key_domain if key_domain is not None else rows
    return [RelSpec(rows, [("mod", d), ("mod", d), ("hi32",)]) for _ in range(n_rels)]


def make_relations(specs: list[RelSpec], seed: int) -> list[list[np.ndarray]]:
    return [[column(seed, r, c, s.rows, k) for c, k in enumerate(s.kinds)] for r, s in enumerate(specs)]


def write_relation(path: str, cols: list[np.ndarray]) -> None:
    rows = len(cols[0]) if cols else 0
    with open(path, "wb") as f:
        np.array([rows, len(cols)], dtype=np.uint64).tofile(f)
        for c in cols:
            np.ascontiguousarray(c, dtype=np.uint64).tofile(f)


def read_relation(path: str) -> list[np.ndarray]:
    m = np.fromfile(path, dtype=np.uint64)
    rows, ncols = int(m[0]), int(m[1])
    return [m[2 + j * rows: 2 + (j + 1) * rows] for j in range(ncols)]


def write_dataset(dirpath: str, rels: list[list[np.ndarray]]) -> list[str]:
    os.makedirs(dirpath, exist_ok=True)
    paths = []
    for i, cols in enumerate(rels):
        p = os.path.join(dirpath, f"r{i}")
        write_relation(p, cols)
        paths.append(p)
    return paths


def protocol_input(paths: list[str], queries: str) -> str:
    """stdin for the reference protocol: paths, Done, query lines (main/queries_main.c)."""
    q = queries if queries.endswith("\n") or not queries else queries + "\n"
    return "".join(p + "\n" for p in paths) + "Done\n" + q


# ---- C4: SIGMOD-2018-style batch ------------------------------------------------
C4_SEED = 4
C4_RELS = 14
C4_QUERIES = 1000
C4_BATCH = 50


def c4_spec(scale: float = 1.0, seed: int = C4_SEED) -> list[RelSpec]:
    """14 relations, sizes log-uniform in [1e5, 1e7] x scale, 2..6 columns.  Column roles by
    position: 0, 1, 4 join keys ("mod", D) with D = 1e7 x scale shared by every relation (so any
    key column joins any other with ~n1*n2/D output rows); 2, 5 uniform u32 payloads ("hi32");
    3 a coarser key ("mod", D / 10).  scale = 0.01 is the rand-invariance-gate size."""
    rng = np.random.default_rng(seed)
    d = max(1, int(round(1e7 * scale)))
    role = [("mod", d), ("mod", d), ("hi32",), ("mod", max(1, d // 10)), ("mod", d), ("hi32",)]
    specs = []
    for _ in range(C4_RELS):
        rows = int(round(10 ** rng.uniform(5.0, 7.0) * scale))
        ncols = int(rng.integers(2, 7))
        specs.append(RelSpec(max(1, rows), role[:ncols]))
    return specs


def c4_queries(specs: list[RelSpec], n: int = C4_QUERIES, seed: int = C4_SEED) -> list[str]:
    """SIGMOD-style queries: 2-4 bindings, chain or star equi-joins on key columns, 0-2 filters
    on u32 payload columns (scale-free selectivity), 1-3 selects."""
    rng = np.random.default_rng(seed + 1000)
    out = []
    for _ in range(n):
        nb = int(rng.integers(2, 5))
        rels = [int(x) for x in rng.choice(len(specs), nb, replace=False)]
        keys = [[c for c, k in enumerate(specs[r].kinds) if k[0] == "mod"] for r in rels]
        pays = [[c for c, k in enumerate(specs[r].kinds) if k[0] == "hi32"] for r in rels]
        star = rng.random() < 0.35
        preds = []
        for b in range(1, nb):
            a = 0 if star else b - 1
            preds.append(f"{a}.{int(rng.choice(keys[a]))}={b}.{int(rng.choice(keys[b]))}")
        nf = int(rng.choice([0, 1, 2], p=[0.3, 0.45, 0.25]))
        for _ in range(nf):
            cands = [b for b in range(nb) if pays[b]]
            if not cands:
                break
            b = int(rng.choice(cands))
            op = ">" if rng.random() < 0.5 else "<"
            v = int(rng.integers(1 << 28, (1 << 32) - (1 << 28)))
            preds.append(f"{b}.{int(rng.choice(pays[b]))}{op}{v}")
        rng.shuffle(preds)
        ns = int(rng.integers(1, 4))
        sels = []
        for _ in range(ns):
            b = int(rng.integers(0, nb))
            sels.append(f"{b}.{int(rng.integers(0, len(specs[rels[b]].kinds)))}")
        out.append(" ".join(map(str, rels)) + "|" + "&".join(preds) + "|" + " ".join(sels) + "\n")
    return out


def c4_batches(queries: list[str], batch: int = C4_BATCH) -> str:
    """the query lines in batches of <= `batch`, each batch closed by an F line"""
    text = []
    for i in range(0, len(queries), batch):
        text.extend(queries[i:i + batch])
        text.append("F\n")
    return "".join(text)


# ---- C5: skewed 2-relation join --------------------------------------------------
C5_SEED = 5
C5_ROWS = 1_000_000_000
C5_THETA = 0.9
C5_PERM_SEED = 55
C5_QUERY = "0 1|0.1=1.0|0.2 1.2\n"
# C5 at its own size (C5_ROWS per side): the printed bytes and the pair count, pinned against the
# key-range-sharded aggregate truth by tests/test_gpu_fullsize_batch.py (print_sums,
# src/utilities.c:216-219, over the join of src/join.c:325-392); benchmarks/c5.py checks its
# line against them in-run
C5_1E9_STDOUT = "896635233956162571 9653025849244459604 \n"
C5_1E9_PAIRS = 384016487678819


def c5_spec(rows: int = C5_ROWS, theta: float = C5_THETA, domain: int | None = None) -> list[RelSpec]:
    """r0 = (v % N, Zipf key, u32 payload), r1 = (Zipf key, v % N, u32 payload): both Zipf columns
    over D = N (default) share one rank->key permutation, so the heavy ranks collide."""
    d = domain if domain is not None else rows
    z = ("zipf", d, theta, C5_PERM_SEED)
    return [RelSpec(rows, [("mod", rows), z, ("hi32",)]), RelSpec(rows, [z, ("mod", rows), ("hi32",)])]


# ---- device-side generation of the bench workloads (libqe's generator, bit-exact with the above) --
def gen_c4(ctx, scale: float = 1.0) -> list[RelSpec]:
    """the 14 C4 relations generated in HBM by libqe (qe_gen_relation)"""
    specs = c4_spec(scale)
    for r, sp in enumerate(specs):
        ctx.gen_relation(sp.rows, sp.kinds, seed=C4_SEED, gen_rel=r)
    ctx.sync()
    return specs


def gen_c5(ctx, rows: int, row_start: int = 0, total_rows: int | None = None) -> list[RelSpec]:
    """relations r0, r1 of c5_spec(total_rows) -- rows [row_start, row_start + rows) of each --
    generated in HBM.  The Zipf CDF is built by libqe in a fixed summation order: the same keys on
    every run."""
    n = total_rows or rows
    specs = c5_spec(n)
    ctx.set_zipf(n, C5_THETA, C5_PERM_SEED)
    try:
        for r, sp in enumerate(specs):
            ctx.gen_relation(rows, sp.kinds, seed=C5_SEED, gen_rel=r, row_start=row_start)
    finally:
        ctx.set_zipf_table(0, 0, 0)
    return specs

