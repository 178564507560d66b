"""The multi-GPU half of the C ABI on one MI355X: an RCCL communicator of one rank (qe_comm_init),
the all-reduce and the exchange through it, and the partitioned executor qe_run_queries_dist on
every golden of the real reference -- queries in the plan's domain run partitioned, the others on
the faithful executor, and the bytes must be the reference's either way.  (RCCL refuses two ranks
on one device, so N > 1 runs on the driver's 8-GPU node; the same C plan runs at world 2 and 3
under gloo in tests/test_plan_gloo.py.)"""
import ctypes as C
import json

import numpy as np
import pytest

import goldens
from qe import datagen as dg
from qe import lib

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def comm(ctx):
    c = lib.Comm(ctx, 1, 0, lib.comm_unique_id())
    yield c
    c.close()


def test_allreduce_one_rank_is_exact(ctx, comm):
    v = [1, (1 << 64) - 1, 5, 1 << 63]
    assert comm.allreduce(v) == v


def test_shuffle_one_rank_keeps_every_row(ctx, comm):
    rng = np.random.default_rng(7)
    n = 300_007
    k = rng.integers(0, 1 << 62, n, dtype=np.uint64)
    a = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
    b = np.arange(n, dtype=np.uint32)
    P = ctx.pairs_from_host(k, a)
    L = ctx.list_from_host(b)
    ok, (oa, ob), on = comm.shuffle(P.key, n, [P.val, L.d])
    assert on == n
    kk, aa = np.empty(n, np.uint64), np.empty(n, np.uint32)
    Q = lib.Pairs()
    Q.key, Q.val, Q.n = ok, oa, n
    ctx._chk(ctx.lib.qe_pairs_to_host(ctx.h, C.byref(Q), kk.ctypes.data, aa.ctypes.data))
    M = lib.List()
    M.d, M.n = ob, n
    bb = ctx.list_to_host(M)
    # the rows travel whole: b is the original position, so (k, a) must be the row it names
    assert np.array_equal(np.sort(bb), b)
    assert np.array_equal(kk, k[bb]) and np.array_equal(aa, a[bb])
    for p in (ok, oa, ob):
        ctx.buffer_free(p)
    ctx.pairs_free(P)
    ctx.list_free(L)
    x, sent = comm.stats()
    assert x >= 1 and sent == 0          # one rank: everything stays home


_loaded = {"key": None}


def _load(ctx, ds):
    key = json.dumps(ds, sort_keys=True)
    if _loaded["key"] != key:
        ctx.drop_relations()
        rels, _ = goldens.dataset(ds)
        for cols in rels:
            ctx.load_relation(cols)
        _loaded["key"] = key


@pytest.mark.parametrize("fixture", [f.split("/")[-1][:-5] for f in goldens.golden_files()])
def test_dist_executor_matches_every_golden(ctx, comm, fixture):
    doc = goldens.load(f"{goldens.GOLDEN_DIR}/{fixture}.json")
    _load(ctx, doc["dataset"])
    planned = 0
    for case in doc["cases"]:
        for cm in (comm, None):
            out, rc, refused = ctx.run_dist(case["input"], cm)
            assert (out, rc) == (case["stdout"], case["rc"]), (case["input"], cm is None)
        planned += refused == 0
    if fixture in ("c4", "fuzz_a", "headline"):
        assert planned >= len(doc["cases"]) // 2     # most of them really ran partitioned


def test_dist_executor_aggregate_fallback_on_every_golden(ctx, comm):
    """materialisation limit 0: a planned join too large to materialise (QE_ETOOBIG) sends its query
    to the faithful executor, which takes the aggregate form where the reference's output allows
    it and fails loudly where it does not -- never a different answer (C5's shape at 1e9 rows)"""
    ctx.set_materialize_limit(0)
    ran = 0
    try:
        for name, idx, ds, case in goldens.all_cases(include_headline=False):
            _load(ctx, ds)
            try:
                out, rc, _ = ctx.run_dist(case["input"], comm)
            except lib.QEError as e:
                assert e.code == lib.QE_ETOOBIG, (name, idx, str(e))
                continue
            assert (out, rc) == (case["stdout"], case["rc"]), (name, idx, case["input"])
            ran += 1
    finally:
        ctx.set_materialize_limit(0x7FFFFFFF)
        ctx.drop_relations()
        _loaded["key"] = None
    assert ran > 100


@pytest.mark.slow
def test_dist_executor_c3_100m_one_rank(ctx, comm):
    """the partitioned plan at the headline size through a one-rank RCCL communicator equals the
    faithful executor (itself pinned to the aggregate truth by test_gpu_fullsize)"""
    N = 100_000_000
    q = "0 1 2 3|0.1=1.0&1.1=2.0&2.1=3.0&3.2>1000000000&3.2<3000000000|1.2 2.2 3.2\n"
    ctx.drop_relations()
    _loaded["key"] = None
    try:
        kinds = [("mod", N), ("mod", N), ("hi32",)]
        for r in range(4):
            ctx.gen_relation(N, kinds, seed=1, gen_rel=r)
        want, _ = ctx.run(q)
        rows = ctx.last_result_rows()
        out, rc, refused = ctx.run_dist(q, comm)
        assert (out, rc, refused) == (want, 0, 0)
        assert ctx.last_result_rows() == rows
    finally:
        ctx.drop_relations()


def _carry_launches(ctx, q, comm):
    ctx.set_profiling(True)
    ctx.reset_stats()
    out, rc, refused = ctx.run_dist(q, comm)
    n = ctx.kernel_stats().get("sort_pass_carry", {}).get("launches", 0)
    ctx.set_profiling(False)
    return out, rc, refused, n


@pytest.mark.slow
def test_dist_executor_carries_bindings_through_the_join(ctx, comm):
    """joins whose derived side carries two and three bindings (C3's chain) at 75 M rows, where that
    side (> 2^25 rows after the filter) is sorted by the lookback-free two-level sort: its extra
    bindings ride through the sort and the bucket join (sort_pass_carry launches), and the printed
    bytes equal the faithful executor's"""
    N = 75_000_001
    ctx.drop_relations()
    _loaded["key"] = None
    try:
        kinds = [("mod", N), ("mod", N), ("hi32",)]
        for r in range(4):
            ctx.gen_relation(N, kinds, seed=3, gen_rel=r)
        qs = ("0 1 2 3|0.1=1.0&1.1=2.0&2.1=3.0&3.2>1000000000&3.2<3000000000|1.2 2.2 3.2\n",
              "0 1 2 3|0.1=1.0&1.1=2.0&2.1=3.0&3.2>2000000000|3.0 1.2 2.1\n",
              "3 2 1 0|0.0=1.1&1.0=2.1&2.0=3.1&0.2<3000000000|0.2 1.2 2.2\n",
              "0 1 2 3|0.1=1.0&1.1=2.0&2.1=3.0&3.2>1000000000|0.2 1.2 2.2 3.2\n")
        planned = 0
        for q in qs:
            want, _ = ctx.run(q)
            out, rc, refused, carried = _carry_launches(ctx, q, comm)
            assert (out, rc) == (want, 0), q
            if refused == 0:                  # planned (the last one's binding 0 list is not relational)
                planned += 1
                assert carried > 0, q
        assert planned >= 2
    finally:
        ctx.drop_relations()


@pytest.mark.slow
def test_dist_executor_carry_falls_back_on_a_skewed_bucket(ctx, comm):
    """a derived side whose key has one heavy value (a bucket beyond LDS): the carry join gives the
    inputs back and the join runs on positions with takes -- same bytes as the faithful executor"""
    N = 50_000_003
    rng = np.random.default_rng(11)
    ctx.drop_relations()
    _loaded["key"] = None
    try:
        rels = []
        for r in range(4):
            c0 = rng.integers(0, N, N, dtype=np.uint64)
            if r == 1:
                c0[rng.random(N) < 0.05] = 12345           # ~1.7 M rows share one key
            rels.append([c0, rng.integers(0, N, N, dtype=np.uint64), rng.integers(0, 1 << 32, N, dtype=np.uint64)])
        for cols in rels:
            ctx.load_relation(cols)
        q = "0 1 2 3|0.1=1.0&1.1=2.0&2.1=3.0&3.2>1000000000|1.2 2.2 3.2\n"
        want, _ = ctx.run(q)
        out, rc, refused, _ = _carry_launches(ctx, q, comm)
        assert (out, rc, refused) == (want, 0, 0)
    finally:
        ctx.drop_relations()


@pytest.mark.slow
def test_dist_executor_last_join_in_aggregate_form(ctx, comm, monkeypatch):
    """C3's last join only feeds the checksums: the engine's join_sums returns its pair count and
    the selects' sums without materialising the pairs (bucket_join_sums), and a filtered binding
    read only by selects of one column carries that column's values instead of its rowids --
    the same bytes as the faithful executor, as the materialised last join (QE_PLAN_AGG=0) and as
    rowids throughout (QE_PLAN_VALUES=0), and the same row count"""
    N = 75_000_001
    ctx.drop_relations()
    _loaded["key"] = None
    try:
        kinds = [("mod", N), ("mod", N), ("hi32",)]
        for r in range(4):
            ctx.gen_relation(N, kinds, seed=5, gen_rel=r)
        qs = ("0 1 2 3|0.1=1.0&1.1=2.0&2.1=3.0&3.2>1000000000&3.2<3000000000|1.2 2.2 3.2\n",
              "0 1 2 3|0.1=1.0&1.1=2.0&2.1=3.0&3.2>2000000000|3.2 3.2 1.0 2.1\n",
              "0 1|0.1=1.0&1.2>3000000000|1.2 1.0\n")
        for q, want_agg in zip(qs, (1, 1, None)):   # (the last one's side is below the carry sort's size)
            want, _ = ctx.run(q)
            rows = ctx.last_result_rows()
            ctx.set_profiling(True)
            ctx.reset_stats()
            out, rc, refused = ctx.run_dist(q, comm)
            agg = ctx.kernel_stats().get("bucket_join_sums", {}).get("launches", 0)
            ctx.set_profiling(False)
            assert (out, rc, refused) == (want, 0, 0), q
            assert ctx.last_result_rows() == rows, q
            assert want_agg is None or agg == want_agg, q
            for knob in ("QE_PLAN_AGG", "QE_PLAN_VALUES", "QE_SCAN_VALUES"):   # materialised last join;
                # rowids, not values; values gathered after the scan, not emitted by it
                monkeypatch.setenv(knob, "0")
                out0, rc0, _ = ctx.run_dist(q, comm)
                monkeypatch.delenv(knob)
                assert (out0, rc0) == (want, 0), (q, knob)
    finally:
        ctx.drop_relations()
