"""qe_join_pairs -- the partitioned plan's join: both sides sorted by their two global radix passes
only, then each 15-bit bucket joined in LDS (bucket_join, csrc/qe_sort.hip) -- against numpy: the
multiset of (R val, S val) pairs must be exactly the equi-join's (join_relations,
src/join.c:325-392, emits every matching pair once; the plan needs no order).  Covers both forms of
the deferred two-level sort (lookback and lookback-free: below / from 2^22 rows), base columns (rowids
generated) and gathered lists, fan-out above 1 (the optimistic buffers outgrown: exact re-run),
two sides of different key bounds (both sorted over the union bounds: one bucket geometry), and
every fallback to the ordinary sort + merge (an in-bucket domain beyond LDS, skewed buckets, small
inputs)."""
import numpy as np
import pytest

from qe import lib

pytestmark = pytest.mark.gpu


def _ref(rk, rv, sk, sv):
    """sorted array of packed (rval << 32 | sval) over every matching pair"""
    so = np.argsort(sk, kind="stable")
    sks, svs = sk[so], sv[so]
    lo = np.searchsorted(sks, rk, "left")
    hi = np.searchsorted(sks, rk, "right")
    cnt = (hi - lo).astype(np.int64)
    P = int(cnt.sum())
    off = np.concatenate([[0], np.cumsum(cnt)[:-1]])
    r = np.repeat(rv, cnt).astype(np.uint64)
    s = svs[np.arange(P, dtype=np.int64) + np.repeat(lo - off, cnt)].astype(np.uint64)
    return np.sort((r << np.uint64(32)) | s)


def _check(ctx, rk, sk, gathered=True, expect=None, stage=None):
    n_r, n_s = len(rk), len(sk)
    ctx.drop_relations()
    relR = ctx.load_relation([rk])
    relS = ctx.load_relation([sk])
    rows = np.random.default_rng(n_r).permutation(n_r).astype(np.uint32)
    lst = ctx.list_from_host(rows)
    R = ctx.gather_pairs(ctx.column(relR, 0), lst if gathered else None)
    S = ctx.gather_pairs(ctx.column(relS, 0), None)
    ctx.set_profiling(True)
    ctx.reset_stats()
    a, b = ctx.join_pairs(R, S)
    stats = ctx.kernel_stats()
    launched = stats.get("bucket_join", {}).get("launches", 0)
    ctx.set_profiling(False)
    got = np.sort((ctx.list_to_host(a).astype(np.uint64) << np.uint64(32)) | ctx.list_to_host(b).astype(np.uint64))
    rv = rows if gathered else np.arange(n_r, dtype=np.uint32)
    want = _ref(rk[rv] if gathered else rk, rv, sk, np.arange(n_s, dtype=np.uint32))
    np.testing.assert_array_equal(got, want)
    for x in (a, b):
        ctx.list_free(x)
    ctx.pairs_free(R)
    ctx.pairs_free(S)
    ctx.list_free(lst)
    ctx.drop_relations()
    if expect is not None:
        assert (launched > 0) == expect, launched
    if stage is not None:
        assert stats.get(stage, {}).get("launches", 0) > 0, sorted(stats)
    return len(want)


@pytest.mark.parametrize("n", [(1 << 25) + 777, 3_000_001])      # lookback-free / lookback two-level form
def test_bucket_join_uniform(ctx, n):
    rng = np.random.default_rng(n)
    rk = rng.integers(0, n, n, dtype=np.uint64)
    sk = rng.integers(0, n, n // 2 + 1, dtype=np.uint64)
    _check(ctx, rk, sk, gathered=True, expect=True)


def test_bucket_join_segments_beyond_one_pass2_tile(ctx):
    """lookback-free form with the first-pass digits skewed 3:1 (buckets stay small): a second-pass
    segment then holds ~12 K words, more than one 9216-word sub-tile, so pass 2 walks a segment in
    sub-tiles with running digit offsets (uniform keys never do: ~8192 +- 90 words)"""
    rng = np.random.default_rng(29)
    n = (1 << 22) + 777   # the lookback-free form from 2^22 keys; a full group's segments average 8 K words

    def keys(m):
        p = np.where(np.arange(256) < 128, 1.5, 0.5)
        d1 = rng.choice(256, m, p=p / p.sum()).astype(np.uint64)
        d2 = rng.integers(0, 128, m, dtype=np.uint64)
        low = rng.integers(0, 1 << 10, m, dtype=np.uint64)
        return (((d2 << np.uint64(8)) | d1) << np.uint64(10)) | low   # 25 varying bits, L = 10

    rk, sk = keys(n), keys(n // 2 + 3)
    _check(ctx, rk, sk, gathered=True, expect=True)
    _check(ctx, rk, sk, gathered=False, expect=True)


def test_bucket_join_base_columns_and_fanout(ctx):
    """both sides base columns (rowids generated); ~4 partners per row: the optimistic nR + nS
    buffers are outgrown and the kernel re-runs with the exact size"""
    n = 4_000_003
    rng = np.random.default_rng(3)
    d = 1 << 20                                                           # 20 varying bits, ~4 rows a key
    rk = rng.integers(0, d, n, dtype=np.uint64) | np.uint64(1 << 22)     # constant bit: kconst path
    sk = rng.integers(0, d, n, dtype=np.uint64) | np.uint64(1 << 22)
    P = _check(ctx, rk, sk, gathered=False, expect=True)
    assert P > 2 * n


@pytest.mark.parametrize("n_small", [40_000, 700_001])
def test_join_small_side_against_a_big_one(ctx, n_small):
    """a side too small for the deferred two-level sort joined with a big one (the big side's
    deferred sort completes, the merge joins them; forcing the small side into the bucket geometry
    measured slower on C4, profiles/r03_c4_hjsmall_ab.log)"""
    rng = np.random.default_rng(n_small)
    n = 3_000_000
    rk = rng.integers(0, n, n, dtype=np.uint64)
    sk = rng.integers(0, n, n_small, dtype=np.uint64)
    _check(ctx, rk, sk, gathered=True, expect=False)
    _check(ctx, sk, rk, gathered=True, expect=False)   # the small side as R


@pytest.mark.parametrize("shape", ["different_bounds", "wide_domain", "skewed", "small"])
def test_bucket_join_fallbacks(ctx, shape):
    rng = np.random.default_rng(7)
    n = 3_000_000
    if shape == "different_bounds":       # R varies in 22 bits, S in 23: both sorted over the union bounds
        rk = rng.integers(0, 1 << 22, n, dtype=np.uint64)
        sk = rng.integers(0, 1 << 23, n, dtype=np.uint64)
    elif shape == "wide_domain":          # 30 varying bits: 15 left inside a bucket, beyond LDS
        rk = rng.integers(0, 1 << 30, n, dtype=np.uint64)
        sk = np.concatenate([rk[: n // 2], rng.integers(0, 1 << 30, n // 2, dtype=np.uint64)])
    elif shape == "skewed":               # one key holds a third of the rows: its bucket is beyond LDS
        rk = rng.integers(0, 1 << 24, n, dtype=np.uint64)
        rk[: n // 3] = 12345
        sk = rng.integers(0, 1 << 24, n, dtype=np.uint64)
        sk[:10] = 12345
    else:
        rk = rng.integers(0, 5000, 4000, dtype=np.uint64)
        sk = rng.integers(0, 5000, 3000, dtype=np.uint64)
    if shape == "skewed":   # the join launches, flags the bucket, and the sides complete by LSD passes
        _check(ctx, rk, sk, gathered=True, expect=True, stage="sort_pass_skew")
    elif shape == "different_bounds":   # one geometry for both (unify_geometry): the bucket join runs
        _check(ctx, rk, sk, gathered=True, expect=True)
    else:
        _check(ctx, rk, sk, gathered=True, expect=False)


def test_bucket_join_long_chain_in_one_bucket_is_linear(ctx):
    """~3000 equal keys on BOTH sides of one bucket that still fits LDS (9 M pairs from one key):
    the chain join would emit each pair k links down the chain (quadratic: minutes in one
    workgroup); a chain past HJ_CHAIN_MAX flags the bucket and the sorts + merge join take it"""
    rng = np.random.default_rng(11)
    n = 3_000_000
    rk = rng.integers(0, 1 << 24, n, dtype=np.uint64)
    sk = rng.integers(0, 1 << 24, n, dtype=np.uint64)
    rk[:3000] = 12345
    sk[:3000] = 12345
    # the path taken, not the wall time: the bucket join ran, flagged the long chain
    # and the sorts + merge join took the join (its kernel ran: stage mj_fused)
    P = _check(ctx, rk, sk, gathered=True, expect=True, stage="mj_fused")
    assert P >= 9_000_000


def test_bucket_join_materialisation_limit(ctx):
    n = 3_000_000
    rng = np.random.default_rng(9)
    rk = rng.integers(0, n, n, dtype=np.uint64)
    ctx.set_materialize_limit(1000)
    try:
        with pytest.raises(lib.QEError) as e:
            _check(ctx, rk, rk.copy(), gathered=False)
        assert e.value.code == lib.QE_ETOOBIG
    finally:
        ctx.set_materialize_limit(0x7FFFFFFF)
        ctx.drop_relations()
