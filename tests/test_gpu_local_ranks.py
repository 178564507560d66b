"""The multi-GPU data path with W > 1 ranks on the one MI355X of the box: qe_run_queries_local runs
qe_run_queries_dist on W in-process ranks (worker contexts of one GPU, one host thread each) over
the in-process transport of qe_comm_init_local -- only the communicator's three RCCL operations are
replaced (counts all-to-all, grouped send/recv, all-reduce); the partitioning, the per-peer
offsets, qe_bucket_select with W > 1, the plan and every kernel are the production code.
References: the batch loop src/utilities.c:289-300, the join src/join.c:325-392 and print_sums
src/utilities.c:197-224 -- the printed bytes must be the reference's at every W."""
import re

import pytest

import goldens
from qe import lib

pytestmark = pytest.mark.gpu

C3 = "0 1 2 3|0.1=1.0&1.1=2.0&2.1=3.0&3.2>1000000000&3.2<3000000000|1.2 2.2 3.2\n"
WELL_FORMED = re.compile(r"[0-9 ]+\|[0-9.=<>&]+\|[0-9. ]+\n")


def _load(ctx, ds):
    ctx.drop_relations()
    rels, _ = goldens.dataset(ds)
    for cols in rels:
        ctx.load_relation(cols)


@pytest.mark.parametrize("world,bcast", [(2, "0"), (3, "0"), (8, "0"), (2, "2"), (3, "2"), (8, "1")])
@pytest.mark.parametrize("fixture", [f.split("/")[-1][:-5] for f in goldens.golden_files()])
def test_local_ranks_match_every_golden(ctx, fixture, world, bcast, monkeypatch):
    """every golden at W ranks: exit-0 well-formed queries as one batch (one line per query, so the
    batch's bytes are the concatenation), the others one by one; rows really moved between ranks.
    QE_PLAN_BCAST: 0 every join partitioned, 2 every join of a derived side with a whole base
    relation broadcast (the derived side stays, the whole column joins it), 1 the cost model"""
    monkeypatch.setenv("QE_PLAN_BCAST", bcast)
    doc = goldens.load(f"{goldens.GOLDEN_DIR}/{fixture}.json")
    _load(ctx, doc["dataset"])
    batch = [c for c in doc["cases"] if c["rc"] == 0 and WELL_FORMED.fullmatch(c["input"])]
    alone = [c for c in doc["cases"] if c not in batch]
    sent = 0
    if batch:
        out, rc, refused, b = ctx.run_local("".join(c["input"] for c in batch), world)
        sent += b
        want = "".join(c["stdout"] for c in batch)
        if out != want:                                   # name the first query that differs
            for c in batch:
                assert ctx.run_local(c["input"], world)[:2] == (c["stdout"], 0), c["input"]
        assert (out, rc) == (want, 0)
        if fixture in ("c4", "fuzz_a", "headline"):
            assert refused <= len(batch) // 2             # most of them ran partitioned
    for c in alone:
        out, rc, _, b = ctx.run_local(c["input"], world)
        sent += b
        assert (out, rc) == (c["stdout"], c["rc"]), c["input"]
    if fixture in ("c4", "fuzz_a", "headline") and bcast == "0":
        assert sent > 0                                   # derived join sides crossed ranks


def test_one_rank_too_large_stops_every_rank(ctx, monkeypatch):
    """a join past the materialisation limit on ONE rank only: every rank leaves the planned query
    together (one all-reduce), the query re-runs on rank 0's faithful executor, the bytes are the
    reference's; nobody waits in a later exchange"""
    monkeypatch.setenv("QE_PLAN_BCAST", "0")
    doc = goldens.load(f"{goldens.GOLDEN_DIR}/headline.json")
    _load(ctx, doc["dataset"])
    case = next(c for c in doc["cases"] if c["input"] == C3)
    ws = ctx.workers(2)
    ctx.lib.qe_set_materialize_limit(ws[1].h, 100)
    g = lib.LocalComms(ws)
    try:
        res = g.run(C3)
        assert g.bytes_sent() > 0
    finally:
        g.close()
        ctx.lib.qe_set_materialize_limit(ws[1].h, 0x7FFFFFFF)
    assert res[0] == (case["stdout"], 0, 1), res[0]       # refused once: the faithful fallback
    assert res[1][1] == 0


def test_limit_bounds_the_global_pair_count(ctx):
    """the limit bounds a join's pair count summed over the ranks (the reference's DArray holds the
    whole result): a limit each rank's share fits under but the total does not still sends the
    query to the faithful executor, as on one rank"""
    doc = goldens.load(f"{goldens.GOLDEN_DIR}/headline.json")
    _load(ctx, doc["dataset"])
    q = "0 1|0.1=1.0|0.2 1.2\n"
    want, _ = ctx.run(q)
    pairs = ctx.last_result_rows()
    assert pairs > 1000
    ctx.set_materialize_limit(pairs * 2 // 3)
    try:
        out1, rc1, ref1 = ctx.run_dist(q)                  # one rank: planned join too large
        out2, rc2, ref2, _ = ctx.run_local(q, 2)           # two ranks: each share below the limit
    finally:
        ctx.set_materialize_limit(0x7FFFFFFF)
    # the fallback's faithful executor takes the aggregate form or fails; never different bytes
    assert (ref1, ref2) == (1, 1)
    assert (out1, rc1) == (out2, rc2)


@pytest.mark.slow
@pytest.mark.parametrize("world", [2, 8])
def test_local_ranks_c3_100m(ctx, world):
    """the headline query at its size (4 x 100 M rows) on W in-process ranks: the faithful
    executor's bytes (pinned to the aggregate truth by test_gpu_fullsize), the same row count, no
    fallback; at 8 ranks the three derived sides exchanged, at 2 the cost model's broadcast joins
    (no derived side moves: each rank joins its rows with the whole base columns)"""
    N = 100_000_000
    ctx.drop_relations()
    try:
        kinds = [("mod", N), ("mod", N), ("hi32",)]
        for r in range(4):
            ctx.gen_relation(N, kinds, seed=1, gen_rel=r)
        want, _ = ctx.run(C3)
        rows = ctx.last_result_rows()
        out, rc, refused, sent = ctx.run_local(C3, world)
        assert (out, rc, refused) == (want, 0, 0)
        assert ctx.last_result_rows() == rows
        assert (sent > 0) == (world == 8)
    finally:
        ctx.drop_relations()


@pytest.mark.parametrize("world", [2, 3])
def test_exchange_sends_u32_keys_when_they_fit(ctx, world, monkeypatch):
    """keys below 2^32 cross ranks as 4 B (QE_EXCHANGE_K32, default on): the same bytes printed as
    with 8-B keys, fewer bytes sent -- C3's exchanged sides carry a key + 1-2 rowid/value columns,
    so 8 + 4c -> 4 + 4c bytes a row (the receiver's sort takes the u32 keys as they arrive)"""
    monkeypatch.setenv("QE_PLAN_BCAST", "0")
    doc = goldens.load(f"{goldens.GOLDEN_DIR}/headline.json")
    _load(ctx, doc["dataset"])
    case = next(c for c in doc["cases"] if c["input"] == C3)
    monkeypatch.setenv("QE_EXCHANGE_K32", "0")
    out64, rc64, _, sent64 = ctx.run_local(C3, world)
    monkeypatch.setenv("QE_EXCHANGE_K32", "1")
    out32, rc32, _, sent32 = ctx.run_local(C3, world)
    assert (out64, rc64) == (case["stdout"], 0)
    assert (out32, rc32) == (case["stdout"], 0)
    assert 0 < sent32 < sent64
    assert sent32 <= sent64 * 3 // 4 + 1               # at least a key's 4 B of every 16-B row
