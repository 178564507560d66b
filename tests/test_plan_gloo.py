"""The C partitioned plan (include/qe_plan.h, host/qe_plan.c) on CPU: the same compiled plan that
drives libqe + RCCL on the GPUs, over a numpy engine (tests/plan_engine.py) -- one rank here, and
world_size 2 and 3 under torch.distributed gloo.

* Domain check: every golden of the real reference either is refused (QE_ENOTSUP, the faithful
  executor runs it) or comes out byte-identical -- W-class (positional garbage) outputs included.
* Sharding: N ranks print what one rank prints, and C3 equals the aggregate truth."""
import numpy as np
import pytest
import torch.multiprocessing as mp

import goldens
import plan_engine as pe
from qe import datagen as dg

QE_ENOTSUP = -6
C3 = "0 1 2 3|0.1=1.0&1.1=2.0&2.1=3.0&3.2>1000000000&3.2<3000000000|1.2 2.2 3.2\n"


def _run_world(rels, queries, world, limits=None, global_limit=None, opts=None):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = pe.free_port()
    procs = [ctx.Process(target=pe.worker, args=(r, world, port, rels, queries, q, limits, global_limit, opts))
             for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=600)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    return res


@pytest.mark.parametrize("optional", ["all", "none"])
@pytest.mark.parametrize("fixture", [f.split("/")[-1][:-5] for f in goldens.golden_files()])
def test_every_golden_is_refused_or_exact(fixture, optional):
    """with the engine's optional entries (scan2: a fused scan + refine; join_carry: a side's
    extra bindings delivered by the join; join_sums: the last join's checksums without its
    pairs; column / keys_of: a base relation's next join key riding with its rows) and without
    them (a scan then a refine; takes; a materialised last join; gathered keys)"""
    doc = goldens.load(f"{goldens.GOLDEN_DIR}/{fixture}.json")
    rels, _ = goldens.dataset(doc["dataset"])
    on = optional == "all"
    eng = pe.NumpyPlanEngine(rels, 0, 1, fused_scan=on, join_carry=on, join_sums=on, values=on, join_agg=on,
                             key_carry=on)
    accepted = {"T": 0, "W": 0}
    for c in doc["cases"]:
        out, rc, _, _ = eng.run(c["input"])
        if rc == QE_ENOTSUP:
            continue
        assert rc == 0, (c["input"], rc)
        assert (out, c["rc"]) == (c["stdout"], 0), c["input"]
        accepted[c.get("class", "T")] = accepted.get(c.get("class", "T"), 0) + 1
    assert eng.live_handles() == 0                     # the plan releases every array it made
    t_cases = sum(c.get("class") == "T" for c in doc["cases"])
    if fixture in ("c4", "fuzz_a", "fuzz_c", "headline"):
        assert accepted["T"] >= 0.75 * t_cases, accepted   # the relational class is the plan's domain
        assert (eng.sums_calls > 0) == on                  # and its last joins take the aggregate form
        assert (eng.values_calls > 0) == on                # and select values ride instead of rowids
    if fixture == "headline" and on:
        assert eng.scan2_values > 0                        # C3's fused scan emits 3.2's values
        assert eng.agg_calls > 0                           # G1/G2: two base relations, aggregate form
        assert eng.keys_of_calls > 0                       # C3: R2's and R1's next join keys rode with them
        assert eng.values_rows > 0                         # ... and their rows as their select column's values


def test_check_names_the_reason():
    rels = dg.make_relations(dg.chain_spec(4, 1000), 1)
    eng = pe.NumpyPlanEngine(rels, 0, 1)
    acc, why = eng.check("0 1|0.2>5&1.2<7&0.1=1.0|0.2\n")      # two filter lists: positional scan_join
    assert acc == [False] and "scan_join" in why
    acc, why = eng.check("0 1|0.1=1.0|0.2 1.2\n0 0|0.1=0.1|0.2\n")
    assert acc == [True, False] and "DO_NOTHING" in why
    acc, _ = eng.check(C3)
    assert acc == [True]


@pytest.mark.parametrize("world", [2, 3])
def test_c3_chain_on_ranks_equals_one_rank_and_truth(world, monkeypatch):
    import agg_truth
    monkeypatch.setenv("QE_PLAN_BCAST", "0")   # the partitioned form of every join (exchanges)
    rows = 60_000
    rels = dg.make_relations(dg.chain_spec(4, rows), 1)
    one = pe.NumpyPlanEngine(rels, 0, 1).run(C3)
    c2 = rels[3][2]
    mask = (c2 > np.uint64(1000000000)) & (c2 < np.uint64(3000000000))
    cnt, nrows, sums = agg_truth.chain4_sums(rels, rows, mask)
    want = f"{cnt}\n" + "".join(f"{s} " for s in sums) + "\n"
    assert one[:3] == (want, 0, nrows)
    res, nex, live = _run_world(rels, [C3, "0 1|0.1=1.0|0.2 1.2\n"], world)
    assert res[0][:3] == (want, 0, nrows)
    pairs_want = agg_truth.pair_sums(rels[0], rels[1], rows)
    assert res[1][0] == f"{pairs_want[1]} {pairs_want[2]} \n"
    # whole base relations are bucketed locally (replicated columns): only derived sides move --
    # C3 reordered (R2-sigma(R3), then R1, then R0): one exchange per join; the 2-rel query none
    assert nex == 3
    assert live == 0


@pytest.mark.parametrize("bcast", ["0", "1", "2"])
def test_two_ranks_match_goldens(bcast, monkeypatch):
    """QE_PLAN_BCAST: 0 every join partitioned (derived sides exchanged), 2 every join of a derived
    side with a whole base relation broadcast (the derived side stays, the base side is the whole
    column), 1 the plan's cost model -- the bytes are the reference's in every form"""
    monkeypatch.setenv("QE_PLAN_BCAST", bcast)
    doc = goldens.load(f"{goldens.GOLDEN_DIR}/fuzz_a.json")
    rels, _ = goldens.dataset(doc["dataset"])
    one = pe.NumpyPlanEngine(rels, 0, 1)
    cases = [c for c in doc["cases"] if one.run(c["input"])[1] == 0][:60]
    res, nex, _ = _run_world(rels, [c["input"] for c in cases], 2)
    assert len(cases) >= 40
    if bcast == "0":
        assert nex > 0
    for c, (out, rc, _, _) in zip(cases, res):
        assert (out, rc) == (c["stdout"], 0), c["input"]


@pytest.mark.parametrize("world", [2, 3])
def test_c3_broadcast_joins(world, monkeypatch):
    """C3 with every join broadcast: R2, R1 and R0 are whole base relations, so no derived side
    moves (0 exchanges) and the output is still the aggregate truth; the cost model picks the
    broadcast form at 2 ranks for C3's shape (one link between two GPUs) and never for a join of
    two derived sides"""
    import agg_truth
    rows = 60_000
    rels = dg.make_relations(dg.chain_spec(4, rows), 1)
    c2 = rels[3][2]
    mask = (c2 > np.uint64(1000000000)) & (c2 < np.uint64(3000000000))
    cnt, nrows, sums = agg_truth.chain4_sums(rels, rows, mask)
    want = f"{cnt}\n" + "".join(f"{s} " for s in sums) + "\n"
    monkeypatch.setenv("QE_PLAN_BCAST", "2")
    res, nex, live = _run_world(rels, [C3], world)
    assert res[0][:3] == (want, 0, nrows)
    assert nex == 0 and live == 0
    monkeypatch.setenv("QE_PLAN_BCAST", "1")
    res, nex, _ = _run_world(rels, [C3], 2)
    assert res[0][:3] == (want, 0, nrows)
    assert nex == 0                                   # the model: broadcast at 2 ranks


def test_one_rank_too_large_stops_every_rank():
    """a join whose bucket is past the materialisation limit on ONE rank only: every rank leaves
    the query with QE_ETOOBIG together (one all-reduce), none waits forever in the next exchange"""
    rows = 20_000
    rels = dg.make_relations(dg.chain_spec(4, rows), 1)
    res, _, _ = _run_world(rels, [C3, "0 1|0.1=1.0|0.2 1.2\n"], 2, limits=[1 << 62, 100], opts={"join_agg": False})
    assert res[0][1] == -5 and res[1][1] == -5
    # the last join of two base relations in aggregate form materialises nothing: no limit applies
    res, _, _ = _run_world(rels, ["0 1|0.1=1.0|0.2 1.2\n"], 2, limits=[1 << 62, 100])
    assert res[0][1] == 0


def test_global_pair_count_is_what_the_limit_bounds():
    """the materialisation limit bounds a join's pair count over ALL ranks (the reference's DArray
    holds the whole result): a limit every rank's share stays under, but the total exceeds, still
    ends the query with QE_ETOOBIG on every rank -- as it does on one rank"""
    rows = 20_000
    rels = dg.make_relations(dg.chain_spec(4, rows), 1)
    q2 = "0 1|0.1=1.0|0.2 1.2\n"
    one = pe.NumpyPlanEngine(rels, 0, 1, join_agg=False)
    out, rc, pairs, _ = one.run(q2)
    assert rc == 0 and pairs > 1000
    limit = pairs * 2 // 3                    # above each of two ranks' ~pairs/2, below the total
    one.set_global_limit(limit)
    assert one.run(q2)[1] == -5
    res, _, _ = _run_world(rels, [q2], 2, global_limit=limit, opts={"join_agg": False})
    assert res[0][1] == -5


def test_ranks_with_different_plan_switches_fail_together(monkeypatch):
    """QE_PLAN_BCAST / QE_DIST_REORDER are read once per query on each rank; a rank whose
    environment differs would broadcast a join its peer exchanges and the collectives would no
    longer pair up (a hang).  The query's first all-reduce carries the switches: every rank fails
    the query with QE_EINVAL together, and the next query (switches agreed) still runs"""
    monkeypatch.delenv("QE_PLAN_BCAST", raising=False)
    rows = 20_000
    rels = dg.make_relations(dg.chain_spec(4, rows), 1)
    q2 = "0 1|0.1=1.0|0.2 1.2\n"
    want = pe.NumpyPlanEngine(rels, 0, 1, join_agg=False).run(q2)[0]
    env = {0: {"QE_PLAN_BCAST": "0"}, 1: {"QE_PLAN_BCAST": "2"}}
    res, _, _ = _run_world(rels, [C3, q2], 2, opts={"env": env, "join_agg": False})
    assert res[0][1] == -1 and res[1][1] == -1
    env = {0: {"QE_DIST_REORDER": "0"}, 1: {"QE_DIST_REORDER": "1"}}
    res, _, _ = _run_world(rels, [C3], 2, opts={"env": env})
    assert res[0][1] == -1
    env = {0: {"QE_PLAN_BCAST": "0"}, 1: {"QE_PLAN_BCAST": "0"}}
    res, _, _ = _run_world(rels, [q2], 2, opts={"env": env, "join_agg": False})
    assert res[0][:2] == (want, 0)
