"""Fused per-bucket sort + merge join (tl_join, csrc/qe_sort.hip; opt-in, QE_FUSED_JOIN=1) at the sizes where qe_sort_pairs
stops before its per-bucket step (two-level sort from 2^25 pairs): the pairs and their order
(key, then R order, then S order -- join_relations, src/join.c:342-377), R's match counts and
rowids, the driver counts that join_payloads consumes, the fallback when the output outgrows
nR + nS, and the aggregate (QE_ETOOBIG) path.  Checked against a vectorised numpy restatement of
the reference merge on stably sorted inputs."""
import numpy as np
import pytest

from qe import lib

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _fused_on(monkeypatch):
    monkeypatch.setenv("QE_FUSED_JOIN", "1")   # opt-in path (off by default: measured slower)

N = (1 << 25) + 777


def _ref_pairs(rk, rv, sk, sv):
    ro = np.argsort(rk, kind="stable")
    so = np.argsort(sk, kind="stable")
    rks, rvs, sks, svs = rk[ro], rv[ro], sk[so], sv[so]
    lo = np.searchsorted(sks, rks, "left")
    hi = np.searchsorted(sks, rks, "right")
    cnt = (hi - lo).astype(np.int64)
    off = np.concatenate([[0], np.cumsum(cnt)[:-1]])
    P = int(cnt.sum())
    out_r = np.repeat(rvs, cnt)
    out_s = svs[np.arange(P, dtype=np.int64) + np.repeat(lo - off, cnt)]
    return out_r, out_s, cnt.astype(np.uint32), rks, rvs


def _sides(ctx, rkeys, skeys, rows_r):
    """R: gathered from a loaded column through a rowid list (vals = rowids); S: a base column
    (rowids generated).  Both carry their column's load-time bounds: same bucket geometry."""
    relR = ctx.load_relation([rkeys])
    relS = ctx.load_relation([skeys])
    lst = ctx.list_from_host(rows_r)
    R = ctx.gather_pairs(ctx.column(relR, 0), lst)
    S = ctx.gather_pairs(ctx.column(relS, 0), None)
    return R, S, lst


def _launches(ctx, name):
    return ctx.kernel_stats().get(name, {}).get("launches", 0)


def test_fused_join_pairs_match_and_driver_counts(ctx):
    rng = np.random.default_rng(11)
    colR = rng.integers(0, N, N, dtype=np.uint64)
    sk = rng.integers(0, N, N, dtype=np.uint64)
    rows = rng.permutation(N).astype(np.uint32)
    ctx.set_profiling(True)
    ctx.reset_stats()
    R, S, lst = _sides(ctx, colR, sk, rows)
    ctx.sort_pairs(R)
    ctx.sort_pairs(S)
    a, b = ctx.merge_join(R, S)
    assert _launches(ctx, "tl_join") == 1 and _launches(ctx, "mj_fused") == 0
    e_r, e_s, e_cnt, rks, rvs = _ref_pairs(colR[rows], rows, sk, np.arange(N, dtype=np.uint32))
    np.testing.assert_array_equal(ctx.list_to_host(a), e_r)
    np.testing.assert_array_equal(ctx.list_to_host(b), e_s)
    np.testing.assert_array_equal(ctx.counts_to_host(R.match, N), e_cnt)
    d = ctx.driver_counts(R, S, a, b, 0, N)          # S rowids distinct: counts from R's match counts
    want = np.zeros(N, dtype=np.uint32)
    want[rvs] = e_cnt
    np.testing.assert_array_equal(ctx.counts_to_host(d, N), want)
    ctx.counts_free(d)
    assert _launches(ctx, "sort_local") == 0          # R's rowids came from the fused join itself
    gk, gv = ctx.pairs_to_host(R)                     # completes the deferred sort: sorted keys
    np.testing.assert_array_equal(gk, rks)
    np.testing.assert_array_equal(gv, rvs)
    gk, gv = ctx.pairs_to_host(S)
    np.testing.assert_array_equal(gk, np.sort(sk, kind="stable"))
    for x in (a, b):
        ctx.list_free(x)
    ctx.pairs_free(R)
    ctx.pairs_free(S)
    ctx.list_free(lst)
    ctx.set_profiling(False)


def test_fused_join_output_beyond_optimistic_buffers(ctx):
    """every key three times on each side: 1.5 x (nR + nS) pairs -- the fused join finds it does
    not fit and the merge runs as usual on the completed sorts"""
    rng = np.random.default_rng(12)
    distinct = rng.choice(1 << 26, N // 3 + 1, replace=False).astype(np.uint64)
    colR = rng.permutation(np.repeat(distinct, 3)[:N])
    sk = rng.permutation(np.repeat(distinct, 3)[:N])
    rows = np.arange(N, dtype=np.uint32)[::-1].copy()
    ctx.set_profiling(True)
    ctx.reset_stats()
    R, S, lst = _sides(ctx, colR, sk, rows)
    ctx.sort_pairs(R)
    ctx.sort_pairs(S)
    a, b = ctx.merge_join(R, S)
    assert _launches(ctx, "tl_join") == 1
    e_r, e_s, e_cnt, _, _ = _ref_pairs(colR[rows], rows, sk, np.arange(N, dtype=np.uint32))
    assert a.n == len(e_r) > 2 * N
    np.testing.assert_array_equal(ctx.list_to_host(a), e_r)
    np.testing.assert_array_equal(ctx.list_to_host(b), e_s)
    for x in (a, b):
        ctx.list_free(x)
    ctx.pairs_free(R)
    ctx.pairs_free(S)
    ctx.list_free(lst)
    ctx.set_profiling(False)


def test_fused_join_too_big_to_materialise_then_counts(ctx):
    rng = np.random.default_rng(13)
    colR = rng.integers(0, N, N, dtype=np.uint64)
    sk = rng.integers(0, N, N, dtype=np.uint64)
    rows = rng.permutation(N).astype(np.uint32)
    R, S, lst = _sides(ctx, colR, sk, rows)
    ctx.sort_pairs(R)
    ctx.sort_pairs(S)
    ctx.set_materialize_limit(1000)
    try:
        with pytest.raises(lib.QEError) as ei:
            ctx.merge_join(R, S)
        assert ei.value.code == lib.QE_ETOOBIG
        P = ctx.merge_join_counts(R, S)
    finally:
        ctx.set_materialize_limit(0x7FFFFFFF)
    e_r, _, e_cnt, _, _ = _ref_pairs(colR[rows], rows, sk, np.arange(N, dtype=np.uint32))
    assert P == len(e_r)
    np.testing.assert_array_equal(ctx.counts_to_host(R.match, N), e_cnt)
    ctx.pairs_free(R)
    ctx.pairs_free(S)
    ctx.list_free(lst)
