"""qe_join_aggregate -- the aggregate form of the last join of two base columns (C5, csrc/qe_agg.hip):
pair count and both weighted checksums from value-carrying sorts and one merge-path counting pass,
against numpy (every row's partner count by searchsorted, sums wrapped mod 2^64).  Shapes: uniform
keys, heavy keys whose runs cross many tiles on one or both sides, keys with constant bits, one
side without a value column, disjoint key sets, empty sides, and the refusals (values >= 2^32,
keys varying in more than 32 bits).  The executor's use of it is pinned by the goldens in mode
agg0 (tests/test_gpu_golden.py) and by C5 at 1e9 rows (tests/test_gpu_fullsize_batch.py)."""
import numpy as np
import pytest

from qe import lib

pytestmark = pytest.mark.gpu


def _truth(kR, vR, kS, vS):
    sS = np.sort(kS)
    sR = np.sort(kR)
    cS = (np.searchsorted(sS, kR, "right") - np.searchsorted(sS, kR, "left")).astype(np.uint64)
    cR = (np.searchsorted(sR, kS, "right") - np.searchsorted(sR, kS, "left")).astype(np.uint64)
    with np.errstate(over="ignore"):
        pairs = int(np.sum(cS, dtype=np.uint64))
        a = int(np.sum(cS * vR.astype(np.uint64), dtype=np.uint64)) if vR is not None else 0
        b = int(np.sum(cR * vS.astype(np.uint64), dtype=np.uint64)) if vS is not None else 0
    return pairs, a, b


def _run(ctx, kR, vR, kS, vS):
    ctx.drop_relations()
    rR = ctx.load_relation([kR] + ([vR] if vR is not None else []))
    rS = ctx.load_relation([kS] + ([vS] if vS is not None else []))
    got = ctx.join_aggregate(ctx.column(rR, 0), ctx.column(rR, 1) if vR is not None else None,
                             ctx.column(rS, 0), ctx.column(rS, 1) if vS is not None else None)
    ctx.drop_relations()
    return got


def _heavy(rng, n, domain, heavy_frac, nheavy=3):
    k = rng.integers(0, domain, n, dtype=np.uint64)
    m = rng.random(n) < heavy_frac
    k[m] = rng.integers(0, nheavy, int(m.sum()), dtype=np.uint64) * np.uint64(7919) + np.uint64(11)
    return k


@pytest.mark.parametrize("shape", ["uniform", "heavy_both", "heavy_one", "const_bits", "no_val_s", "disjoint",
                                   "tiny", "one_key", "small_uniform", "wide_domain", "zipf"])
def test_join_aggregate_matches_numpy(ctx, shape):
    """from 2^22 rows in total with 16..30 varying key bits the bucketed form runs (two partition
    passes per side, LDS counting, giant buckets on many workgroups), below it the sort + merge-path
    form (small_uniform, tiny, one_key)"""
    rng = np.random.default_rng(len(shape))
    nR, nS, dom = 3_000_017, 2_000_003, 1 << 22
    if shape == "small_uniform":
        nR, nS = 1_000_003, 900_001
        kR = rng.integers(0, dom, nR, dtype=np.uint64)
        kS = rng.integers(0, dom, nS, dtype=np.uint64)
    elif shape == "wide_domain":         # 30 varying bits: 2^15 values per bucket, mostly empty
        kR = rng.integers(0, 1 << 30, nR, dtype=np.uint64)
        kS = rng.integers(0, 1 << 30, nS, dtype=np.uint64)
        kS[::3] = kR[: len(kS[::3])]     # a third of S joins
    elif shape == "zipf":                # a C5-like head: many giant buckets, light keys in between
        kR = (rng.zipf(1.4, nR).astype(np.uint64) * np.uint64(2654435761)) % np.uint64(1 << 28)
        kS = (rng.zipf(1.4, nS).astype(np.uint64) * np.uint64(2654435761)) % np.uint64(1 << 28)
    elif shape == "uniform":
        kR = rng.integers(0, dom, nR, dtype=np.uint64)
        kS = rng.integers(0, dom, nS, dtype=np.uint64)
    elif shape == "heavy_both":          # runs of ~10^5 rows: every heavy key crosses many tiles
        kR = _heavy(rng, nR, dom, 0.3)
        kS = _heavy(rng, nS, dom, 0.2)
    elif shape == "heavy_one":
        kR = _heavy(rng, nR, dom, 0.5, nheavy=1)
        kS = rng.integers(0, dom, nS, dtype=np.uint64)
        kS[:5] = 11                      # five partners of the heavy R key
    elif shape == "const_bits":          # bit 40 set everywhere, bits 0-2 zero: the field is shifted
        kR = (rng.integers(0, 1 << 20, nR, dtype=np.uint64) << np.uint64(3)) | np.uint64(1 << 40)
        kS = (rng.integers(0, 1 << 20, nS, dtype=np.uint64) << np.uint64(3)) | np.uint64(1 << 40)
    elif shape == "no_val_s":
        kR = rng.integers(0, 1 << 16, nR, dtype=np.uint64)
        kS = rng.integers(0, 1 << 16, nS, dtype=np.uint64)
    elif shape == "disjoint":            # R even, S odd keys: no pair
        kR = rng.integers(0, dom, nR, dtype=np.uint64) * np.uint64(2)
        kS = rng.integers(0, dom, nS, dtype=np.uint64) * np.uint64(2) + np.uint64(1)
    elif shape == "tiny":
        nR, nS = 5, 3
        kR = np.array([4, 1, 4, 9, 4], dtype=np.uint64)
        kS = np.array([4, 9, 4], dtype=np.uint64)
    else:                                # every key equal: P = nR * nS, the field is empty
        nR, nS = 70_001, 50_003
        kR = np.full(nR, 123456789, dtype=np.uint64)
        kS = np.full(nS, 123456789, dtype=np.uint64)
    vR = rng.integers(0, 1 << 32, nR, dtype=np.uint64)
    vS = None if shape == "no_val_s" else rng.integers(0, 1 << 32, nS, dtype=np.uint64)
    assert _run(ctx, kR, vR, kS, vS) == _truth(kR, vR, kS, vS)


def test_join_aggregate_empty_side(ctx):
    ctx.drop_relations()
    r = ctx.load_relation([np.arange(10, dtype=np.uint64), np.arange(10, dtype=np.uint64)])
    empty = lib.Col(ctx.column(r, 0).d, 0)
    assert ctx.join_aggregate(ctx.column(r, 0), ctx.column(r, 1), empty, None) == (0, 0, 0)
    assert ctx.join_aggregate(empty, None, ctx.column(r, 0), ctx.column(r, 1)) == (0, 0, 0)
    ctx.drop_relations()


@pytest.mark.parametrize("what", ["wide_values", "wide_keys"])
def test_join_aggregate_refuses(ctx, what):
    rng = np.random.default_rng(5)
    n = 1000
    k = rng.integers(0, 1 << 10, n, dtype=np.uint64)
    v = rng.integers(0, 1 << 32, n, dtype=np.uint64)
    if what == "wide_values":
        v[7] = 1 << 32
    else:
        k[3] = 1 << 40
    ctx.drop_relations()
    r = ctx.load_relation([k, v])
    with pytest.raises(lib.QEError) as e:
        ctx.join_aggregate(ctx.column(r, 0), ctx.column(r, 1), ctx.column(r, 0), ctx.column(r, 1))
    assert e.value.code == lib.QE_ENOTSUP
    ctx.drop_relations()
