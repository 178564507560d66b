"""C5 skew path on the GPU: the device Zipf generator, the
aggregate form of the merge join (qe_merge_join_counts + qe_checksum_weighted), the
materialisation limit (QE_ETOOBIG), and the executor's aggregate fallback -- all through the
C ABI, checked against numpy restatements, the reference's golden vectors and, at 1e8 rows,
the aggregate push-down truth of tests/agg_truth.py."""
import numpy as np
import pytest

import agg_truth
import goldens
from qe import datagen as dg
from qe import lib

pytestmark = pytest.mark.gpu

DEFAULT_LIMIT = 0x7FFFFFFF


def _cdf_on_device(cdf: np.ndarray):
    import torch
    t = torch.from_numpy(np.ascontiguousarray(cdf)).cuda()
    torch.cuda.synchronize()
    return t


@pytest.mark.parametrize("domain,theta,rows", [(20000, 0.9, 200_000), (100_003, 0.9, 300_000),
                                               (3000, 1.2, 50_000), (1 << 20, 0.7, 400_000), (1, 0.9, 1000)])
def test_device_zipf_matches_numpy(ctx, domain, theta, rows):
    """kind 2 with the numpy CDF table: the same keys, bit for bit (guide-table search and the
    Feistel permutation are exact integer/IEEE-compare work)"""
    cdf = dg.zipf_cdf(domain, theta)
    t = _cdf_on_device(cdf)
    ctx.drop_relations()
    ctx.set_zipf_table(t.data_ptr(), domain, dg.C5_PERM_SEED)
    kind = ("zipf", domain, theta, dg.C5_PERM_SEED)
    rel = ctx.gen_relation(rows, [kind, ("hi32",)], seed=dg.C5_SEED, gen_rel=1, row_start=12345)
    want = dg.column(dg.C5_SEED, 1, 0, rows, kind, start=12345)
    got = ctx.column_to_host(rel, 0)
    assert np.array_equal(got, want)
    ctx.set_zipf_table(0, 0, 0)
    ctx.drop_relations()


def test_zipf_without_table_fails_loudly(ctx):
    ctx.set_zipf_table(0, 0, 0)
    with pytest.raises(lib.QEError):
        ctx.gen_relation(10, [("zipf", 100, 0.9, 1)], seed=1, gen_rel=0)


def _skewed(rng, n, domain, heavy):
    k = rng.integers(0, domain, n).astype(np.uint64)
    k[rng.random(n) < heavy] = np.uint64(domain // 2)
    return k


def _np_counts(rk, sk):
    """per-row partner counts and the pair count, numpy"""
    ss = np.sort(sk)
    rs = np.sort(rk)
    cR = np.searchsorted(ss, rk, "right") - np.searchsorted(ss, rk, "left")
    cS = np.searchsorted(rs, sk, "right") - np.searchsorted(rs, sk, "left")
    return cR.astype(np.uint64), cS.astype(np.uint64), int(cR.sum())


@pytest.mark.parametrize("nR,nS,domain,heavy", [(100_000, 80_000, 50_000, 0.3), (3, 200_000, 10, 0.0),
                                                (250_000, 1, 7, 0.5), (70_000, 90_000, 1 << 40, 0.2)])
def test_merge_join_counts_and_weighted_checksum(ctx, nR, nS, domain, heavy):
    rng = np.random.default_rng(nR + nS)
    rk, sk = _skewed(rng, nR, domain, heavy), _skewed(rng, nS, domain, heavy)
    rv = rng.permutation(nR).astype(np.uint32)
    sv = rng.permutation(nS).astype(np.uint32)
    colR = rng.integers(0, 1 << 63, nR, dtype=np.uint64)
    colS = rng.integers(0, 1 << 63, nS, dtype=np.uint64)
    cR, cS, P = _np_counts(rk, sk)
    R = ctx.sort_pairs(ctx.pairs_from_host(rk, rv))
    S = ctx.sort_pairs(ctx.pairs_from_host(sk, sv))
    assert ctx.merge_join_counts(R, S) == P
    # the materialised join's checksums equal the weighted sums of its sides
    with np.errstate(over="ignore"):
        wantR = int(np.sum(colR[rv] * cR, dtype=np.uint64))
        wantS = int(np.sum(colS[sv] * cS, dtype=np.uint64))
    assert ctx.checksum_weighted(_col(ctx, colR), R) == wantR
    assert ctx.checksum_weighted(_col(ctx, colS), S) == wantS
    if P < 20_000_000:
        a, b = ctx.merge_join(R, S)
        assert a.n == P
        assert ctx.checksum(_col(ctx, colR), a) == wantR
        assert ctx.checksum(_col(ctx, colS), b) == wantS
        ctx.list_free(a)
        ctx.list_free(b)
    ctx.pairs_free(R)
    ctx.pairs_free(S)
    ctx.drop_relations()


def _col(ctx, arr):
    rel = ctx.load_relation([arr])
    return ctx.column(rel, 0)


def _vec_merge(rk, rv, sk, sv):
    """the merge's output for sorted inputs (key, R order, S order), vectorised numpy"""
    lo = np.searchsorted(sk, rk, side="left")
    hi = np.searchsorted(sk, rk, side="right")
    c = hi - lo
    outR = np.repeat(rv, c)
    starts = np.repeat(lo - np.concatenate([[0], np.cumsum(c)[:-1]]), c)
    outS = sv[starts + np.arange(c.sum())]
    return outR.astype(np.uint32), outS.astype(np.uint32)


@pytest.mark.parametrize("shape", ["exact_path", "two_pass_path", "many_heavy"])
def test_heavy_tiles_are_emitted_in_parallel_and_in_order(ctx, shape):
    """tiles over MJ_HEAVY_DEFER (2^20) pairs are expanded by mj_heavy_prep/mj_heavy_emit:
    the output must still be the reference's order (key, R order, S order), on the single-pass
    path (P <= |R| + |S|) and on the two-pass fallback"""
    rng = np.random.default_rng(7)
    if shape == "exact_path":      # one heavy tile, P well under |R| + |S|
        rk = np.concatenate([np.full(2048, 7), rng.integers(10, 1 << 40, 3_000_000)])
        sk = np.concatenate([np.full(600, 7), rk[2048:]])
    elif shape == "two_pass_path":  # P >> |R| + |S|
        rk = np.concatenate([np.full(5000, 7), rng.integers(10, 1000, 20000)])
        sk = np.concatenate([np.full(1000, 7), rng.integers(10, 1000, 20000)])
    else:                            # several heavy keys spread over many tiles
        rk = rng.choice(np.array([3, 5, 9, 11], dtype=np.uint64), 40000)
        sk = rng.choice(np.array([3, 5, 9, 12], dtype=np.uint64), 8000)
    rk, sk = rk.astype(np.uint64), sk.astype(np.uint64)
    rv = rng.permutation(len(rk)).astype(np.uint32)
    sv = rng.permutation(len(sk)).astype(np.uint32)
    R = ctx.sort_pairs(ctx.pairs_from_host(rk, rv))
    S = ctx.sort_pairs(ctx.pairs_from_host(sk, sv))
    a, b = ctx.merge_join(R, S)
    rks, rvs = ctx.pairs_to_host(R)
    sks, svs = ctx.pairs_to_host(S)
    wa, wb = _vec_merge(rks, rvs, sks, svs)
    assert a.n == len(wa)
    assert np.array_equal(ctx.list_to_host(a), wa)
    assert np.array_equal(ctx.list_to_host(b), wb)
    for x in (a, b):
        ctx.list_free(x)
    ctx.pairs_free(R)
    ctx.pairs_free(S)


def test_materialise_limit_and_46bit_overflow(ctx):
    """one key on both sides, 1e7 rows each: P = 1e14 > 2^46 (the lookback field width) -- the
    merge must report the exact count with QE_ETOOBIG, and the count pass must agree"""
    n = 10_000_000
    k = np.full(n, 42, dtype=np.uint64)
    v = np.arange(n, dtype=np.uint32)
    R = ctx.sort_pairs(ctx.pairs_from_host(k, v))
    S = ctx.sort_pairs(ctx.pairs_from_host(k, v))
    a, b = lib.List(), lib.List()
    rc = ctx.lib.qe_merge_join(ctx.h, lib.C.byref(R), lib.C.byref(S), lib.C.byref(a), lib.C.byref(b))
    assert rc == lib.QE_ETOOBIG
    assert a.n == n * n and b.n == n * n and not a.d
    assert ctx.merge_join_counts(R, S) == n * n
    col = np.arange(n, dtype=np.uint64) * np.uint64(3) + np.uint64(1)
    with np.errstate(over="ignore"):
        want = int(np.sum(col, dtype=np.uint64) * np.uint64(n))
    assert ctx.checksum_weighted(_col(ctx, col), R) == want
    # under the limit the same join materialises
    ctx.set_materialize_limit(n * n)
    small_k = k[:1000]
    R2 = ctx.sort_pairs(ctx.pairs_from_host(small_k, v[:1000]))
    S2 = ctx.sort_pairs(ctx.pairs_from_host(small_k, v[:1000]))
    a2, b2 = ctx.merge_join(R2, S2)
    assert a2.n == 1_000_000
    ctx.set_materialize_limit(DEFAULT_LIMIT)
    for p in (R, S, R2, S2):
        ctx.pairs_free(p)
    ctx.list_free(a2)
    ctx.list_free(b2)
    ctx.drop_relations()


_loaded = {"key": None}


def _load(ctx, ds):
    import json
    key = json.dumps(ds, sort_keys=True)
    if _loaded["key"] != key:
        ctx.drop_relations()
        rels, _ = goldens.dataset(ds)
        for cols in rels:
            ctx.load_relation(cols)
        _loaded["key"] = key


def test_executor_aggregate_form_on_every_golden(ctx):
    """materialisation limit 0: every sorted join with a pair takes the aggregate form where
    the executor allows it (nothing later reads its lists) and fails loudly (QE_ETOOBIG)
    where it does not -- never a different answer.  The C5 fixtures must all run."""
    _loaded["key"] = None
    ran = {}
    ctx.set_materialize_limit(0)
    try:
        for name, idx, ds, case in goldens.all_cases(include_headline=False):
            _load(ctx, ds)
            try:
                out, rc = ctx.run(case["input"])
            except lib.QEError as e:
                assert e.code == lib.QE_ETOOBIG, (name, idx, str(e))
                continue
            assert (out, rc) == (case["stdout"], case["rc"]), (name, idx, case["input"])
            ran[name] = ran.get(name, 0) + 1
    finally:
        ctx.set_materialize_limit(DEFAULT_LIMIT)
        ctx.drop_relations()
        _loaded["key"] = None
    c5 = goldens.load(goldens.GOLDEN_DIR + "/c5.json")
    multi = [c for c in c5["cases"] if c["input"].startswith("0 1 2|")]
    assert ran.get("c5", 0) == len(c5["cases"]) - len(multi)
    assert ran.get("c5_theta12", 0) == 3


def test_qe_set_zipf_is_deterministic_and_close_to_numpy(ctx):
    """the libqe-built table (fixed summation order): two builds draw identical keys; against
    the numpy table (sequential float sums) at most a few boundary draws may differ"""
    d, rows = 1 << 20, 1_000_000
    kind = ("zipf", d, 0.9, dg.C5_PERM_SEED)
    got = []
    for _ in range(2):
        ctx.drop_relations()
        ctx.set_zipf(d, 0.9, dg.C5_PERM_SEED)
        rel = ctx.gen_relation(rows, [kind], seed=dg.C5_SEED, gen_rel=0)
        ctx.set_zipf_table(0, 0, 0)
        got.append(ctx.column_to_host(rel, 0))
    assert np.array_equal(got[0], got[1])
    want = dg.column(dg.C5_SEED, 0, 0, rows, kind)
    assert np.count_nonzero(got[0] != want) <= rows // 10000
    ctx.drop_relations()


@pytest.mark.slow
def test_c5_shape_100m_against_aggregate_truth(ctx):
    """the C5 query at 1e8 rows per side (P ~ 6.5e12 pairs: far past the limit) through the
    drop-in executor, against numpy aggregate push-down on the same (device-made) columns"""
    N = 100_000_000
    ctx.drop_relations()
    dg.gen_c5(ctx, N)
    out, rc = ctx.run(dg.C5_QUERY)
    assert rc == 0
    R0 = [ctx.column_to_host(0, c) for c in range(3)]
    R1 = [ctx.column_to_host(1, c) for c in range(3)]
    pairs, s0, s1 = agg_truth.pair_sums(R0, R1, N)
    assert pairs > DEFAULT_LIMIT
    assert out == f"{s0} {s1} \n"
    assert ctx.last_result_rows() == pairs
    ctx.drop_relations()
