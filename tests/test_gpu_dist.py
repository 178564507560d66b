"""GPU tests of the multi-GPU plan's primitives (partition, bucket select, heavy stats, slices)
and of the C5 skew path inside the C plan (the engine's aggregate last join: heavy keys split by
row slice, light keys bucketed) through qe_run_queries_local.  The relational plan's GPU tests
are tests/test_gpu_comm.py and tests/test_gpu_local_ranks.py."""
import numpy as np
import pytest
import torch.multiprocessing as mp

import goldens
import gpu_dist_worker
import plan_engine as pe
from qe import datagen as dg

pytestmark = pytest.mark.gpu

@pytest.mark.parametrize("n,parts,ncols", [(0, 2, 1), (1, 8, 2), (100_000, 8, 3), (3_000_001, 5, 1), (4096, 64, 4),
                                           (2_000_000, 1, 0), (777_777, 7, 4)])
def test_partition_groups_rows_by_destination(ctx, n, parts, ncols):
    """every row lands in its destination's segment exactly once, columns riding along (order
    inside a segment is unspecified: the receiver sorts)"""
    import torch
    rng = np.random.default_rng(n)
    keys = rng.integers(0, 1 << 40, n, dtype=np.uint64)
    cols = [rng.integers(0, 1 << 31, n).astype(np.uint32) for _ in range(ncols)]
    dk = torch.from_numpy(keys.view(np.int64)).cuda()
    dc = [torch.from_numpy(c.view(np.int32)).cuda() for c in cols]
    ok = torch.empty(max(1, n), dtype=torch.int64, device="cuda")
    oc = [torch.empty(max(1, n), dtype=torch.int32, device="cuda") for _ in cols]
    torch.cuda.synchronize()
    counts = ctx.partition(dk.data_ptr(), n, [t.data_ptr() for t in dc], parts, ok.data_ptr(),
                           [t.data_ptr() for t in oc])
    dest = pe.part_of(keys, parts).astype(np.int64)
    assert counts == np.bincount(dest, minlength=parts).tolist()
    gk = ok.cpu().numpy()[:n].view(np.uint64)
    gc = [o.cpu().numpy()[:n].view(np.uint32) for o in oc]
    # rows are identified by their index in the input (carried in the first column when present)
    s0 = 0
    for p, cnt in enumerate(counts):
        seg = slice(s0, s0 + cnt)
        s0 += cnt
        want = np.nonzero(dest == p)[0]
        got_rows = sorted(zip(gk[seg].tolist(), *[c[seg].tolist() for c in gc]))
        want_rows = sorted(zip(keys[want].tolist(), *[c[want].tolist() for c in cols]))
        assert got_rows == want_rows


@pytest.mark.parametrize("n,parts,nheavy", [(0, 2, 0), (1, 1, 0), (5, 3, 1), (100_001, 8, 0), (3_000_001, 8, 5),
                                            (2_000_000, 1, 0), (777_777, 64, 20)])
def test_bucket_select_is_the_hash_bucket(ctx, n, parts, nheavy):
    rng = np.random.default_rng(n + parts)
    keys = rng.integers(0, max(1, n // 3), n, dtype=np.uint64) * np.uint64(0x9E3779B1)
    rel = ctx.load_relation([keys])
    heavy = np.unique(keys[:nheavy]) if nheavy else np.zeros(0, np.uint64)
    dest = pe.part_of(keys, parts).astype(np.int64)
    for part in sorted({0, parts - 1, parts // 2}):
        p = ctx.bucket_select(ctx.column(rel, 0), parts, part, heavy)
        k, v = ctx.pairs_to_host(p)
        ctx.pairs_free(p)
        want = np.nonzero((dest == part) & ~np.isin(keys, heavy))[0]
        np.testing.assert_array_equal(np.sort(v), want.astype(np.uint32))   # each row once, no other
        np.testing.assert_array_equal(k, keys[v])
    ctx.drop_relations()


@pytest.mark.parametrize("n,start,end", [(0, 0, 0), (10, 2, 9), (2_500_000, 123, 2_400_000)])
def test_heavy_stats_counts_and_weighted_sums(ctx, n, start, end):
    rng = np.random.default_rng(7 + n)
    keys = rng.zipf(1.3, n).astype(np.uint64) if n else np.zeros(0, np.uint64)
    vals = rng.integers(0, 1 << 63, n, dtype=np.uint64)
    rel = ctx.load_relation([keys, vals])
    heavy = np.array([1, 2, 3, 5, 1 << 40], dtype=np.uint64)
    w = np.array([3, 1 << 62, 7, 0, 9], dtype=np.uint64)
    counts, s = ctx.heavy_stats(ctx.column(rel, 0), start, end, heavy, ctx.column(rel, 1), w)
    kk, vv = keys[start:end], vals[start:end]
    want_c = [int(np.sum(kk == h)) for h in heavy]
    want_s = 0
    for h, wt in zip(heavy.tolist(), w.tolist()):
        want_s = (want_s + int(np.sum(vv[kk == h], dtype=np.uint64)) * wt) % (1 << 64)
    assert counts.tolist() == want_c and s == want_s
    c2, none = ctx.heavy_stats(ctx.column(rel, 0), start, end, heavy)
    assert c2.tolist() == want_c and none is None
    ctx.drop_relations()


def test_filter_scan_range_and_iota(ctx):
    a = dg.column(3, 1, 2, 50_000, ("hi32",))
    rel = ctx.load_relation([a])
    l = ctx.filter_scan_range(ctx.column(rel, 0), 12_345, 40_000, ">", 1 << 31)
    want = np.nonzero(a[12_345:40_000] > np.uint64(1 << 31))[0] + 12_345
    np.testing.assert_array_equal(ctx.list_to_host(l), want.astype(np.uint32))
    i = ctx.iota(7, 1000)
    np.testing.assert_array_equal(ctx.list_to_host(i), np.arange(7, 1007, dtype=np.uint32))


def test_join_indices_and_take(ctx):
    rng = np.random.default_rng(1)
    ka = rng.integers(0, 500, 20_000, dtype=np.uint64)
    kb = rng.integers(0, 500, 30_000, dtype=np.uint64)
    import torch
    ta, tb = torch.from_numpy(ka.view(np.int64)).cuda(), torch.from_numpy(kb.view(np.int64)).cuda()
    torch.cuda.synchronize()
    ia, ib = ctx.join_indices(ta.data_ptr(), len(ka), tb.data_ptr(), len(kb))
    ha, hb = ctx.list_to_host(ia), ctx.list_to_host(ib)
    assert np.all(ka[ha] == kb[hb])
    got = sorted(zip(ha.tolist(), hb.tolist()))
    want = pe.join_local(ka, kb)
    assert got == sorted(zip(want[0].tolist(), want[1].tolist()))
    src = ctx.list_from_host(np.arange(20_000, dtype=np.uint32) * 3)
    t = ctx.take_u32(src.d, ia)
    np.testing.assert_array_equal(ctx.list_to_host(t), ha * 3)


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_skew_join_on_ranks_equals_faithful_executor_on_c5(ctx, world):
    """C5-shaped Zipf data (9 M rows per side: above QE_AGG_MIN = 2^24 rows in total, where the
    aggregate form takes over): the C plan's aggregate last join at W in-process ranks -- heavy keys sampled, counted per row slice and all-reduced, light keys bucketed
    locally -- prints the faithful executor's bytes (its qe_join_aggregate path) for every query"""
    rows = 9_000_000
    queries = ["0 1|0.1=1.0|0.2 1.2\n", "0 1|0.1=1.0|1.2 0.2 0.2 1.2\n", "1 0|0.0=1.1|0.2 1.2\n",
               "0 1|0.1=1.0|0.2\n"]
    ctx.drop_relations()
    try:
        dg.gen_c5(ctx, rows)
        for q in queries:
            want, _ = ctx.run(q)
            pairs = ctx.last_result_rows()
            if world == 1:
                out, rc, refused = ctx.run_dist(q)
            else:
                out, rc, refused, _ = ctx.run_local(q, world)
            assert (out, rc, refused) == (want, 0, 0), (q, world)
            assert ctx.last_result_rows() == pairs
    finally:
        ctx.drop_relations()


@pytest.mark.parametrize("world", [2, 3])
def test_skew_join_on_ranks_matches_c5_goldens(ctx, world):
    """every C5 golden of the real reference at W in-process ranks, bytes and status"""
    doc = goldens.load(f"{goldens.GOLDEN_DIR}/c5.json")
    rels, _ = goldens.dataset(doc["dataset"])
    ctx.drop_relations()
    try:
        for cols in rels:
            ctx.load_relation(cols)
        for c in doc["cases"]:
            out, rc, _, _ = ctx.run_local(c["input"], world)
            assert (out, rc) == (c["stdout"], c["rc"]), c["input"]
    finally:
        ctx.drop_relations()


def test_c4_replicas_two_ranks_share_one_gpu():
    """bench.py --workload c4 at N = 2 (contiguous shares, concurrent lanes per rank, gloo control
    plane) on the one GPU: the joined output is the full-size fixture's, byte for byte"""
    mpc = mp.get_context("spawn")
    q = mpc.Queue()
    port = pe.free_port()
    procs = [mpc.Process(target=gpu_dist_worker.c4_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = q.get(timeout=600)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert res["parity"] is True and res["n_gpus"] == 2
