"""GPU parity of every device primitive (through the C ABI) against numpy restatements of
the reference functions on the same seeded inputs.  Integer work: bit-exact."""
import numpy as np
import pytest

from qe import datagen as dg
from qe import lib

pytestmark = pytest.mark.gpu

OPS = {"=": np.equal, ">": np.greater, "<": np.less}


def _col(ctx, arr):
    rel = ctx.load_relation([arr])
    return ctx.column(rel, 0)


def _ref_merge(rk, rv, sk, sv):
    """join_relations (src/join.c:342-377), the literal loop (valid for unsorted input)."""
    outR, outS = [], []
    pr, s_start = 0, 0
    nR, nS = len(rk), len(sk)
    while pr < nR and s_start < nS:
        ps, flag = s_start, 0
        while ps < nS:
            if rk[pr] < sk[ps]:
                break
            if rk[pr] > sk[ps]:
                ps += 1
                if flag == 0:
                    s_start = ps
            else:
                outR.append(rv[pr])
                outS.append(sv[ps])
                flag = 1
                ps += 1
        pr += 1
    return np.array(outR, dtype=np.uint32), np.array(outS, dtype=np.uint32)


def _vec_merge(rk, rv, sk, sv):
    """Same output for sorted inputs, vectorised (key, R order, S order)."""
    lo = np.searchsorted(sk, rk, side="left")
    hi = np.searchsorted(sk, rk, side="right")
    c = hi - lo
    outR = np.repeat(rv, c)
    starts = np.repeat(lo - np.concatenate([[0], np.cumsum(c)[:-1]]), c)
    outS = sv[starts + np.arange(c.sum())]
    return outR.astype(np.uint32), outS.astype(np.uint32)


def test_gpu_generator_matches_numpy(ctx):
    rows = 1_000_003
    kinds = [("mod", 1_000_000), ("mod", 777), ("hi32",)]
    rel = ctx.gen_relation(rows, kinds, seed=1, gen_rel=2)
    for j, k in enumerate(kinds):
        want = dg.column(1, 2, j, rows, k)
        col = ctx.column(rel, j)
        assert ctx.checksum(col, None) == int(np.sum(want, dtype=np.uint64))
        l = ctx.list_from_host(np.array([0, 1, 2, rows - 1], dtype=np.uint32))
        got = sum(int(want[i]) for i in [0, 1, 2, rows - 1]) & ((1 << 64) - 1)
        assert ctx.checksum(col, l) == got


@pytest.mark.parametrize("n", [0, 1, 7, 4096, 4097, 100_000, 3_000_001])
@pytest.mark.parametrize("op", ["<", ">", "="])
def test_filter_scan(ctx, n, op):
    rng = np.random.default_rng(n + ord(op))
    a = rng.integers(0, 1000, n, dtype=np.uint64)
    col = _col(ctx, a)
    v = 500 if op != "=" else 7
    l = ctx.filter_scan(col, op, v)
    want = np.nonzero(OPS[op](a, np.uint64(v)))[0].astype(np.uint32)
    np.testing.assert_array_equal(ctx.list_to_host(l), want)
    ctx.list_free(l)


@pytest.mark.parametrize("same", [True, False], ids=["one_column", "two_columns"])
@pytest.mark.parametrize("n,start", [(1, 0), (5, 2), (24_577, 0), (3_000_001, 1_234_567)])
def test_filter_scan2_is_scan_then_refine(ctx, n, start, same):
    """the plan's fused scan + refine of one binding: rowids r in [start, n) with both predicates,
    ascending -- what a scan and a refine of its list give"""
    rng = np.random.default_rng(n + start)
    a = rng.integers(0, 1 << 32, n, dtype=np.uint64)
    b = a if same else rng.integers(0, 1000, n, dtype=np.uint64)
    ca = _col(ctx, a)
    cb = ca if same else _col(ctx, b)
    for (o1, v1), (o2, v2) in (((">", 1 << 30), ("<", 3 << 30)), (("=", int(a[-1])), (">", 0)), (("<", 5), ("=", 7))):
        l = ctx.filter_scan2_range(ca, o1, v1, cb, o2, v2, start, n)
        r = np.arange(start, n)
        want = r[OPS[o1](a[start:], np.uint64(v1)) & OPS[o2](b[start:], np.uint64(v2))].astype(np.uint32)
        np.testing.assert_array_equal(ctx.list_to_host(l), want)
        ctx.list_free(l)


@pytest.mark.parametrize("n", [1, 5, 8191, 500_000])
def test_filter_refine_keeps_order(ctx, n):
    rng = np.random.default_rng(n)
    a = rng.integers(0, 1 << 32, 2 * n + 10, dtype=np.uint64)
    col = _col(ctx, a)
    rows = rng.integers(0, len(a), n).astype(np.uint32)    # arbitrary order, duplicates
    l = ctx.list_from_host(rows)
    ctx.filter_refine(col, ">", 1 << 31, l)
    want = rows[a[rows] > np.uint64(1 << 31)]
    np.testing.assert_array_equal(ctx.list_to_host(l), want)


def test_filter_bad_operator_raises(ctx):
    col = _col(ctx, np.arange(10, dtype=np.uint64))
    with pytest.raises(lib.QEError):
        ctx.filter_scan(col, "!", 3)


@pytest.mark.parametrize("n,domain", [(2, 3), (1000, 10), (70_000, 1 << 20), (1_000_000, 1_000_000),
                                      (2_000_000, 1 << 62), (300_000, 1)])
def test_sort_pairs_stable(ctx, n, domain):
    rng = np.random.default_rng(n)
    k = rng.integers(0, domain, n, dtype=np.uint64)
    v = rng.permutation(n).astype(np.uint32)
    p = ctx.pairs_from_host(k, v)
    ctx.sort_pairs(p)
    gk, gv = ctx.pairs_to_host(p)
    order = np.argsort(k, kind="stable")
    np.testing.assert_array_equal(gk, k[order])
    np.testing.assert_array_equal(gv, v[order])
    assert ctx.is_sorted(p)
    ctx.pairs_free(p)


def _keys_for(case, n, rng):
    if case == "27bit":
        return rng.integers(0, 100_000_000, n, dtype=np.uint64)
    if case == "20bit":                       # one local ranking round (L = 5)
        return rng.integers(0, 1 << 20, n, dtype=np.uint64)
    if case == "31bit":                       # L = 16: two full 8-bit local rounds
        return rng.integers(0, 1 << 31, n, dtype=np.uint64)
    if case == "19bit":                       # below the two-level range: plain LSD
        return rng.integers(0, 1 << 19, n, dtype=np.uint64)
    if case == "const_hi":                    # constant high bits restored from the AND
        return (np.uint64(1 << 40) | rng.integers(0, 1 << 25, n, dtype=np.uint64)).astype(np.uint64)
    if case == "stride8":                     # varying bits start at bit 3
        return (rng.integers(0, 1 << 24, n, dtype=np.uint64) << np.uint64(3)).astype(np.uint64)
    if case == "skew":                        # one key holds half the rows: a bucket overflows LDS
        k = rng.integers(0, 100_000_000, n, dtype=np.uint64)
        k[rng.random(n) < 0.5] = 77_777_777
        return k
    raise ValueError(case)


@pytest.mark.parametrize("case", ["27bit", "20bit", "31bit", "19bit", "const_hi", "stride8", "skew"])
def test_sort_pairs_two_level_sizes(ctx, case):
    """n >= 2^22 takes the two-level sort (15 high bits by global passes, the rest in LDS per
    bucket; at 5 M keys its lookback-free form) when 20..31 bits vary; skew or fewer bits fall
    back to the LSD passes."""
    n = 5_000_000
    rng = np.random.default_rng(len(case))
    k = _keys_for(case, n, rng)
    v = rng.permutation(n).astype(np.uint32)
    p = ctx.pairs_from_host(k, v)
    ctx.sort_pairs(p)
    gk, gv = ctx.pairs_to_host(p)
    order = np.argsort(k, kind="stable")
    np.testing.assert_array_equal(gk, k[order])
    np.testing.assert_array_equal(gv, v[order])
    ctx.pairs_free(p)


@pytest.mark.parametrize("case,with_vals", [("27bit", True), ("27bit", False), ("31bit", True), ("skew", True)])
def test_sort_pairs_lookback_free_two_level(ctx, case, with_vals):
    """n >= 2^22 (QE_SORT_PRE_MIN): the two-level sort whose global passes take their offsets from
    the histogram read (per-tile and per-segment digit counts) instead of a lookback; 'skew' runs
    both passes and then falls back to the LSD passes"""
    n = (1 << 25) + 4_321
    rng = np.random.default_rng(99 + len(case))
    k = _keys_for(case, n, rng)
    if with_vals:
        v = rng.permutation(n).astype(np.uint32)
        p = ctx.pairs_from_host(k, v)
    else:
        v = np.arange(n, dtype=np.uint32)
        col = _col(ctx, k)
        p = ctx.gather_pairs(col, None)
    ctx.sort_pairs(p)
    gk, gv = ctx.pairs_to_host(p)
    order = np.argsort(k, kind="stable")
    np.testing.assert_array_equal(gk, k[order])
    np.testing.assert_array_equal(gv, v[order])
    ctx.pairs_free(p)


@pytest.mark.parametrize("n", [2, 64, 1000, 5120, 5121, 70_000, 699_999, 700_001, 1_048_576, 3_000_000])
@pytest.mark.parametrize("case", ["27bit", "31bit", "12bit", "skew"])
@pytest.mark.parametrize("with_vals", [True, False])
def test_sort_pairs_small_and_one_pass_paths(ctx, n, case, with_vals):
    """n <= 5120: one workgroup sorts in LDS (up to 4 rounds of 8 bits); n <= 700 k: one global
    8-bit pass + LDS buckets; then the 15-bit two-level sort; skew falls back to LSD passes"""
    rng = np.random.default_rng(n * 7 + len(case))
    if case == "12bit":
        k = rng.integers(0, 1 << 12, n, dtype=np.uint64)
    else:
        k = _keys_for(case, n, rng)
    if with_vals:
        v = rng.permutation(n).astype(np.uint32)
        p = ctx.pairs_from_host(k, v)
    else:                                      # base column: rowids generated (IN_KIOTA)
        v = np.arange(n, dtype=np.uint32)
        col = _col(ctx, k)
        p = ctx.gather_pairs(col, None)
    ctx.sort_pairs(p)
    gk, gv = ctx.pairs_to_host(p)
    order = np.argsort(k, kind="stable")
    np.testing.assert_array_equal(gk, k[order])
    np.testing.assert_array_equal(gv, v[order])
    ctx.pairs_free(p)


def test_sort_base_column_generates_rowids(ctx):
    a = dg.column(5, 0, 0, 123_457, ("mod", 50_000))
    col = _col(ctx, a)
    p = ctx.gather_pairs(col, None)
    ctx.sort_pairs(p)
    gk, gv = ctx.pairs_to_host(p)
    order = np.argsort(a, kind="stable")
    np.testing.assert_array_equal(gk, a[order])
    np.testing.assert_array_equal(gv, order.astype(np.uint32))


def test_gather_pairs_list_order(ctx):
    a = dg.column(6, 0, 1, 10_000, ("mod", 999))
    col = _col(ctx, a)
    rows = np.random.default_rng(0).integers(0, 10_000, 33_333).astype(np.uint32)
    l = ctx.list_from_host(rows)
    p = ctx.gather_pairs(col, l)
    gk, gv = ctx.pairs_to_host(p)
    np.testing.assert_array_equal(gk, a[rows])
    np.testing.assert_array_equal(gv, rows)


@pytest.mark.parametrize("nR,nS,dom", [(1, 1, 1), (10, 20, 5), (5000, 7000, 3000), (1_000_000, 1_000_000, 1_000_000),
                                       (300_000, 50_000, 40), (100, 200_000, 3), (0, 10, 4), (10, 0, 4)])
def test_merge_join_sorted(ctx, nR, nS, dom):
    rng = np.random.default_rng(nR * 7 + nS)
    rk = np.sort(rng.integers(0, dom, nR, dtype=np.uint64))
    sk = np.sort(rng.integers(0, dom, nS, dtype=np.uint64))
    rv = rng.integers(0, 1 << 31, nR).astype(np.uint32)
    sv = rng.integers(0, 1 << 31, nS).astype(np.uint32)
    R, S = ctx.pairs_from_host(rk, rv), ctx.pairs_from_host(sk, sv)
    a, b = ctx.merge_join(R, S)
    wa, wb = _vec_merge(rk, rv, sk, sv)
    np.testing.assert_array_equal(ctx.list_to_host(a), wa)
    np.testing.assert_array_equal(ctx.list_to_host(b), wb)


def test_merge_join_skewed_window(ctx):
    # one key matching 100k S rows: the S window does not fit LDS -> global-memory search path
    rk = np.array([1, 5, 5, 5, 9], dtype=np.uint64)
    sk = np.sort(np.concatenate([np.full(100_000, 5, np.uint64), np.arange(10, 20, dtype=np.uint64)]))
    rv = np.arange(5, dtype=np.uint32)
    sv = np.arange(len(sk), dtype=np.uint32)
    R, S = ctx.pairs_from_host(rk, rv), ctx.pairs_from_host(sk, sv)
    a, b = ctx.merge_join(R, S)
    wa, wb = _vec_merge(rk, rv, sk, sv)
    np.testing.assert_array_equal(ctx.list_to_host(a), wa)
    np.testing.assert_array_equal(ctx.list_to_host(b), wb)


@pytest.mark.parametrize("seed", range(6))
def test_merge_join_unsorted_matches_reference_loop(ctx, seed):
    rng = np.random.default_rng(seed)
    nR, nS = int(rng.integers(1, 300)), int(rng.integers(1, 300))
    rk = rng.integers(0, 20, nR, dtype=np.uint64)
    sk = rng.integers(0, 20, nS, dtype=np.uint64)
    if seed % 2:
        sk = np.sort(sk)   # one sorted side, one not
    rv = np.arange(nR, dtype=np.uint32)
    sv = np.arange(nS, dtype=np.uint32)
    R, S = ctx.pairs_from_host(rk, rv), ctx.pairs_from_host(sk, sv)
    a, b = ctx.merge_join(R, S)
    wa, wb = _ref_merge(list(rk), list(rv), list(sk), list(sv))
    np.testing.assert_array_equal(ctx.list_to_host(a), wa)
    np.testing.assert_array_equal(ctx.list_to_host(b), wb)


@pytest.mark.parametrize("nR,nS", [(0, 5), (1000, 999), (100_000, 123_456)])
def test_scan_join(ctx, nR, nS):
    rng = np.random.default_rng(nR)
    rk = rng.integers(0, 4, nR, dtype=np.uint64)
    sk = rng.integers(0, 4, nS, dtype=np.uint64)
    rv = rng.integers(0, 1 << 30, nR).astype(np.uint32)
    sv = rng.integers(0, 1 << 30, nS).astype(np.uint32)
    R, S = ctx.pairs_from_host(rk, rv), ctx.pairs_from_host(sk, sv)
    a, b = ctx.scan_join(R, S)
    m = min(nR, nS)
    eq = rk[:m] == sk[:m]
    np.testing.assert_array_equal(ctx.list_to_host(a), rv[:m][eq])
    np.testing.assert_array_equal(ctx.list_to_host(b), sv[:m][eq])


def _ref_nondup_counts(outR, outS, mode, rows):
    seen = set()
    cnt = np.zeros(rows, dtype=np.uint32)
    for r, s in zip(outR.tolist(), outS.tolist()):
        if (r, s) not in seen:
            seen.add((r, s))
            cnt[r if mode == 0 else s] += 1
    return cnt


@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("dupR,dupS", [(False, False), (True, False), (False, True), (True, True)])
def test_driver_counts(ctx, mode, dupR, dupS):
    rng = np.random.default_rng(mode * 4 + dupR * 2 + dupS)
    rows = 3000
    colR = rng.integers(0, 500, rows, dtype=np.uint64)
    colS = rng.integers(0, 500, rows, dtype=np.uint64)
    lr = rng.integers(0, rows, 4000) if dupR else rng.permutation(rows)[:2000]
    ls = rng.integers(0, rows, 4000) if dupS else rng.permutation(rows)[:2500]
    lr, ls = lr.astype(np.uint32), ls.astype(np.uint32)
    LR = ctx.list_from_host(lr, 0 if dupR else lib.LIST_DISTINCT)
    LS = ctx.list_from_host(ls, 0 if dupS else lib.LIST_DISTINCT)
    cR, cS = _col(ctx, colR), _col(ctx, colS)
    R, S = ctx.gather_pairs(cR, LR), ctx.gather_pairs(cS, LS)
    ctx.sort_pairs(R)
    ctx.sort_pairs(S)
    a, b = ctx.merge_join(R, S)
    ha, hb = ctx.list_to_host(a), ctx.list_to_host(b)
    want = _ref_nondup_counts(ha, hb, mode, rows)
    for use_inputs in (True, False):
        d = ctx.driver_counts(R if use_inputs else None, S if use_inputs else None, a, b, mode, rows)
        np.testing.assert_array_equal(ctx.counts_to_host(d, rows), want)
        ctx.counts_free(d)


def _ref_join_payloads(counts, last, edit):
    order = np.argsort(last, kind="stable")
    l, e = last[order], edit[order]
    return np.repeat(e, counts[l]).astype(np.uint32)


@pytest.mark.parametrize("n", [0, 1, 1000, 300_000, 6_000_000])
def test_join_payloads(ctx, n):
    rng = np.random.default_rng(n)
    rows = max(1, n // 2)
    counts = rng.integers(0, 4, rows).astype(np.uint32)
    last = rng.integers(0, rows, n).astype(np.uint32)
    edit = rng.integers(0, 1 << 31, n + 3).astype(np.uint32)
    L, E = ctx.list_from_host(last), ctx.list_from_host(edit)
    dc = ctx.list_from_host(counts)   # any device u32 buffer works as a count array
    out = ctx.join_payloads(dc.d, rows, L, E)
    np.testing.assert_array_equal(ctx.list_to_host(out), _ref_join_payloads(counts, last, edit[:n]))


def test_join_payloads_short_edit_is_error(ctx):
    L = ctx.list_from_host(np.array([0, 1, 2], dtype=np.uint32))
    E = ctx.list_from_host(np.array([5], dtype=np.uint32))
    dc = ctx.list_from_host(np.ones(3, dtype=np.uint32))
    with pytest.raises(lib.QEError):
        ctx.join_payloads(dc.d, 3, L, E)


def test_join_payloads_beyond_the_materialisation_limit_is_etoobig(ctx):
    """an expansion past the limit (the reference's DArray bound, INT32_MAX by default) fails
    cleanly with QE_ETOOBIG before allocating, as the merge join does -- never a hipMalloc abort"""
    n = 1000
    L = ctx.list_from_host(np.arange(n, dtype=np.uint32))
    E = ctx.list_from_host(np.arange(n, dtype=np.uint32))
    dc = ctx.list_from_host(np.full(n, 2, dtype=np.uint32))      # P = 2000
    ctx.set_materialize_limit(1999)
    try:
        with pytest.raises(lib.QEError) as e:
            ctx.join_payloads(dc.d, n, L, E)
        assert e.value.code == lib.QE_ETOOBIG
        with pytest.raises(lib.QEError) as e:
            ctx.join_payloads_multi(dc.d, n, L, [E, E])
        assert e.value.code == lib.QE_ETOOBIG
        ctx.set_materialize_limit(2000)
        assert ctx.join_payloads(dc.d, n, L, E).n == 2000
    finally:
        ctx.set_materialize_limit(0x7FFFFFFF)


@pytest.mark.parametrize("n", [0, 3, 1_000_001])
def test_checksum_wraps_mod_2_64(ctx, n):
    a = np.full(2 * n + 1, (1 << 63) + 12345, dtype=np.uint64)
    col = _col(ctx, a)
    rows = np.random.default_rng(n).integers(0, len(a), n).astype(np.uint32)
    l = ctx.list_from_host(rows)
    assert ctx.checksum(col, l) == int(np.sum(a[rows], dtype=np.uint64))


def test_join_payloads_multi_shares_the_permutation(ctx):
    rng = np.random.default_rng(5)
    rows, n = 5000, 20_000
    counts = rng.integers(0, 3, rows).astype(np.uint32)
    last = rng.integers(0, rows, n).astype(np.uint32)
    edits = [rng.integers(0, 1 << 31, n + k).astype(np.uint32) for k in range(3)]
    L = ctx.list_from_host(last)
    E = [ctx.list_from_host(e) for e in edits]
    dc = ctx.list_from_host(counts)
    outs = ctx.join_payloads_multi(dc.d, rows, L, E)
    for e, o in zip(edits, outs):
        np.testing.assert_array_equal(ctx.list_to_host(o), _ref_join_payloads(counts, last, e[:n]))


def test_column_bits_at_load(ctx):
    a = np.array([0b1010, 0b1110, 0b1011], dtype=np.uint64)
    rel = ctx.load_relation([a, a * 0 + 7])
    assert ctx.column_bits(rel, 0) == (0b1111, 0b1010)
    assert ctx.column_bits(rel, 1) == (7, 7)


@pytest.mark.parametrize("shape", ["random_small_domain", "random_large", "r_ascending", "s_descending",
                                   "all_equal", "r_descending", "s_records_tied", "multi_chunk",
                                   "many_candidates"])
def test_merge_join_unsorted_shapes(ctx, shape):
    """the parallel form of the literal loop on unsorted inputs (prefix maxima + records of S),
    across chunk boundaries of its scans and the degenerate orders"""
    rng = np.random.default_rng(len(shape))
    n = {"random_large": 70_000, "multi_chunk": 70_000, "many_candidates": 200_003}.get(shape, 3000)
    if shape == "random_small_domain":
        rk, sk = rng.integers(0, 50, n, dtype=np.uint64), rng.integers(0, 50, n + 17, dtype=np.uint64)
    elif shape == "random_large":
        rk, sk = rng.integers(0, 1 << 40, n, dtype=np.uint64), rng.integers(0, 1 << 40, n, dtype=np.uint64)
        sk[::97] = rk[::97][: len(sk[::97])]
    elif shape in ("r_ascending", "many_candidates"):   # every R row a candidate: the long count scan
        rk, sk = np.arange(n, dtype=np.uint64), rng.integers(0, n, n, dtype=np.uint64)
    elif shape == "s_descending":
        rk, sk = rng.integers(0, n, n, dtype=np.uint64), np.arange(n, 0, -1).astype(np.uint64)
    elif shape == "all_equal":
        rk, sk = np.full(n, 7, dtype=np.uint64), np.full(500, 7, dtype=np.uint64)
    elif shape == "r_descending":
        rk, sk = np.arange(n, 0, -1).astype(np.uint64), rng.integers(0, n, n, dtype=np.uint64)
    elif shape == "s_records_tied":   # S's running max repeats (ties with the record value)
        sk = np.repeat(np.arange(0, 300, 3, dtype=np.uint64), 30)
        rng.shuffle(sk[:1500])
        rk = rng.integers(0, 300, n, dtype=np.uint64)
    else:                              # prefix maxima across many 4096-element chunks
        rk = np.sort(rng.integers(0, 1000, n, dtype=np.uint64))[::-1].copy()
        rk[::5000] = 999
        sk = rng.integers(0, 1000, n, dtype=np.uint64)
    rv = rng.permutation(len(rk)).astype(np.uint32)
    sv = rng.permutation(len(sk)).astype(np.uint32)
    R, S = ctx.pairs_from_host(rk, rv), ctx.pairs_from_host(sk, sv)
    a, b = ctx.merge_join(R, S)
    wa, wb = _ref_merge(rk.tolist(), rv.tolist(), sk.tolist(), sv.tolist())
    np.testing.assert_array_equal(ctx.list_to_host(a), wa)
    np.testing.assert_array_equal(ctx.list_to_host(b), wb)


def test_merge_fills_match_counts_and_driver_counts_use_them(ctx):
    rng = np.random.default_rng(8)
    colR = rng.integers(0, 300, 4000, dtype=np.uint64)
    colS = rng.integers(0, 300, 3000, dtype=np.uint64)
    cR, cS = _col(ctx, colR), _col(ctx, colS)
    lr = rng.integers(0, 4000, 6000).astype(np.uint32)          # R side with duplicate rowids
    LR = ctx.list_from_host(lr)
    R = ctx.gather_pairs(cR, LR)
    S = ctx.gather_pairs(cS, None)                               # base column: distinct
    assert S.flags & lib.PAIRS_DISTINCT and S.flags & 4          # stats known from load
    ctx.sort_pairs(R)
    ctx.sort_pairs(S)
    a, b = ctx.merge_join(R, S)
    assert R.match
    d = ctx.driver_counts(R, S, a, b, 0, 4000)
    want = _ref_nondup_counts(ctx.list_to_host(a), ctx.list_to_host(b), 0, 4000)
    np.testing.assert_array_equal(ctx.counts_to_host(d, 4000), want)


def test_load_relation_staged_round_trip(ctx):
    """qe_load_relation copies pageable host columns through the pinned staging ring (32 MiB
    slots, several host threads per slot): 9 M rows = 72 MB per column, two full slots and a
    partial one; every value lands, and the load-time OR / AND are those of the column"""
    n = 9_000_001
    rng = np.random.default_rng(5)
    a = rng.integers(0, 1 << 63, n, dtype=np.uint64)
    b = (rng.integers(0, 1 << 20, n, dtype=np.uint64) << np.uint64(4)) | np.uint64(3)
    rel = ctx.load_relation([a, b])
    s0, b0 = ctx.load_stats()
    assert b0 >= 2 * n * 8 and s0 > 0
    for j, want in enumerate((a, b)):
        c = ctx.column(rel, j)
        p = lib.Pairs()
        p.key, p.val, p.match, p.n = c.d, None, None, c.n
        got = np.empty(n, dtype=np.uint64)
        ctx._chk(ctx.lib.qe_pairs_to_host(ctx.h, lib.C.byref(p), got.ctypes.data, None))
        np.testing.assert_array_equal(got, want)
    kor, kand = ctx.column_bits(rel, 1)
    assert kor == int(np.bitwise_or.reduce(b)) and kand == int(np.bitwise_and.reduce(b))


def test_gather_with_histogram_then_sort(ctx):
    """a gathered list of >= 2^25 rowids whose sort is the lookback-free two-level one: the gather
    also builds that sort's histogram (tl_gather_hist_kernel); sorted (key, rowid) must equal the
    stable numpy sort.  A gathered-but-never-sorted side (freed) must leave nothing behind."""
    n = (1 << 25) + 12_345
    rng = np.random.default_rng(21)
    colv = rng.integers(0, 100_000_000, 50_000_000, dtype=np.uint64)
    col = _col(ctx, colv)
    rows = rng.integers(0, len(colv), n, dtype=np.uint32)      # duplicates: fan-out like a join output
    lst = ctx.list_from_host(rows)
    p = ctx.gather_pairs(col, lst)
    ctx.pairs_free(p)                                          # histogram dropped with the keys
    ctx.set_profiling(True)
    ctx.reset_stats()
    p = ctx.gather_pairs(col, lst)
    ctx.sort_pairs(p)
    hist_launches = ctx.kernel_stats().get("sort_hist", {})
    ctx.set_profiling(False)
    gk, gv = ctx.pairs_to_host(p)
    k = colv[rows]
    order = np.argsort(k, kind="stable")
    np.testing.assert_array_equal(gk, k[order])
    np.testing.assert_array_equal(gv, rows[order])
    assert hist_launches.get("alg_bytes", 0) == 0              # the sort read no histogram of its own
    ctx.pairs_free(p)
    ctx.list_free(lst)


@pytest.mark.parametrize("n", [3_000_000, (1 << 25) + 999])
def test_sort_pairs_crowded_buckets(ctx, n):
    """crowded buckets of ~5000 words (the per-bucket LDS sort's capacity is 5120), with the
    two-level sort's lookback (3 M) and lookback-free (2^25) global passes.  (A four-per-CU
    per-bucket variant capped at 4480 words plus a second launch for larger buckets measured
    0.75 ms SLOWER per C3 query, so there is one 5120-word variant.)"""
    rng = np.random.default_rng(n)
    k = rng.integers(0, 1 << 27, n, dtype=np.uint64)      # 27 varying bits: bucket = key >> 12
    for b in (7, 1000, 20000):
        cur = int(np.count_nonzero((k >> np.uint64(12)) == np.uint64(b)))
        extra = 5000 - cur
        idx = rng.choice(n, extra, replace=False)
        k[idx] = (np.uint64(b) << np.uint64(12)) | rng.integers(0, 4096, extra, dtype=np.uint64)
    sizes = np.bincount((k >> np.uint64(12)).astype(np.int64))
    assert 4480 < sizes.max() <= 5120
    v = rng.permutation(n).astype(np.uint32)
    p = ctx.pairs_from_host(k, v)
    ctx.sort_pairs(p)
    gk, gv = ctx.pairs_to_host(p)
    order = np.argsort(k, kind="stable")
    np.testing.assert_array_equal(gk, k[order])
    np.testing.assert_array_equal(gv, v[order])
    ctx.pairs_free(p)


def test_checksums_batched(ctx):
    """qe_checksums: print_sums' select loop with one round trip -- 40 (column, list) pairs (two
    rounds of 32), an empty list, a whole column (no list); every sum mod 2^64 as qe_checksum"""
    rng = np.random.default_rng(31)
    cols = [rng.integers(0, 1 << 64, 50_000, dtype=np.uint64) for _ in range(3)]
    rels = [_col(ctx, c) for c in cols]
    lists, want, hosts = [], [], []
    for k in range(40):
        j = k % 3
        n = 0 if k == 5 else int(rng.integers(1, 20_000))
        rows = rng.integers(0, 50_000, n, dtype=np.uint32)
        hosts.append(ctx.list_from_host(rows))
        lists.append(hosts[-1])
        want.append(int(cols[j][rows].sum(dtype=np.uint64)) if n else 0)
    cc = (lib.Col * 41)(*([rels[k % 3] for k in range(40)] + [rels[0]]))
    lp = (lib.C.POINTER(lib.List) * 41)(*([lib.C.pointer(l) for l in lists] + [lib.C.POINTER(lib.List)()]))
    want.append(int(cols[0].sum(dtype=np.uint64)))
    out = (lib.C.c_uint64 * 41)()
    ctx._chk(ctx.lib.qe_checksums(ctx.h, 41, cc, lp, out))
    assert list(out) == want
    for k in (0, 7, 39):
        assert ctx.checksum(rels[k % 3], lists[k]) == want[k]
    for l in hosts:
        ctx.list_free(l)


@pytest.mark.parametrize("extra", [13, 4096 + 3, 8191])
def test_partial_last_tile_at_the_end_of_exact_allocations(ctx, extra):
    """relations of 2^22 + extra rows (the lookback-free two-level sort's floor, a partial last
    tile): the last tile's masked lanes and its strided buffer loads run past the columns' ends
    into their DALLOC_SLACK (the soffset stride is not range-checked; a static_assert in qe_sort.hip
    keeps every stride below the slack) -- the planned C3 query equals the faithful executor's
    bytes.  (This checks the partial-tile masking; it cannot catch an over-read that stays inside
    the slack.)"""
    rows = (1 << 22) + extra
    q = "0 1 2 3|0.1=1.0&1.1=2.0&2.1=3.0&3.2>1000000000&3.2<3000000000|1.2 2.2 3.2\n"
    ctx.drop_relations()
    try:
        kinds = [("mod", rows), ("mod", rows), ("hi32",)]
        for r in range(4):
            ctx.gen_relation(rows, kinds, seed=3, gen_rel=r)
        want, rc0 = ctx.run(q)
        got, rc, refused = ctx.run_dist(q)
        assert (got, rc, refused) == (want, 0, 0) and rc0 == 0
    finally:
        ctx.drop_relations()
