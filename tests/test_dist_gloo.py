"""The multi-GPU plan (qe.dist) on CPU: world_size 2 under torch.distributed gloo with a numpy
engine.  The plan's output must equal the reference's golden stdout on every relational-class
(T) golden query it accepts, and equal the single-rank run -- the same DistExecutor code that
drives libqe + RCCL on the GPUs."""
import numpy as np
import pytest
import torch.multiprocessing as mp

import dist_cpu_engine as dce
import goldens
from qe import datagen as dg
from qe.dist import DistExecutor, NotSupported, arrange, parse


def _run_world(rels, queries, world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = dce.free_port()
    procs = [ctx.Process(target=dce.worker, args=(r, world, port, rels, queries, q)) for r in range(world)]
    for p in procs:
        p.start()
    res, ex = q.get(timeout=600)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    return res, ex


def _t_cases(name):
    doc = goldens.load(f"{goldens.GOLDEN_DIR}/{name}.json")
    cases = [c for c in doc["cases"] if c["class"] == "T" and c["rc"] == 0
             and len([l for l in c["input"].splitlines() if l.strip() and not l.startswith("F")]) == 1]
    return doc, cases


def test_arrange_matches_reference_quirk_k2():
    # SURVEY.md A.3 example K2: `0 3 1|0.2=13&0.1=1.0&2.0=1.0` runs 2.0=1.0 before 0.1=1.0
    _, preds, _ = parse("0 3 1|0.2=13&0.1=1.0&2.0=1.0|0.2")
    order = [(p.kind, p.a, p.b) for p in arrange(preds)]
    assert order[0][0] == "filter"
    assert order.index(("join", (2, 0), (1, 0))) < order.index(("join", (0, 1), (1, 0)))


@pytest.mark.parametrize("fixture", ["fuzz_a", "known_answers", "protocol"])
def test_single_rank_plan_matches_goldens(fixture):
    doc, cases = _t_cases(fixture)
    rels, _ = goldens.dataset(doc["dataset"])
    eng = dce.NumpyEngine(rels, 0, 1)
    ex = DistExecutor(eng, [len(r[0]) for r in rels])
    checked = 0
    for c in cases:
        line = [l for l in c["input"].splitlines() if l.strip()][0]
        try:
            out, _ = ex.run(line)
        except NotSupported:
            continue
        assert out == c["stdout"], line
        checked += 1
    assert checked >= min(5, len(cases))


def test_two_rank_gloo_plan_matches_goldens():
    doc, cases = _t_cases("fuzz_a")
    rels, _ = goldens.dataset(doc["dataset"])
    lines = [[l for l in c["input"].splitlines() if l.strip()][0] for c in cases][:60]
    res, nex = _run_world(rels, lines, 2)
    assert nex > 0
    checked = 0
    for line, c, (out, _) in zip(lines, cases, res):
        if out.startswith("!"):
            continue
        assert out == c["stdout"], line
        checked += 1
    assert checked >= 30


@pytest.mark.parametrize("world", [2, 3])
def test_c3_chain_two_and_three_ranks(world):
    rows = 60_000
    rels = dg.make_relations(dg.chain_spec(4, rows), 1)
    query = "0 1 2 3|0.1=1.0&1.1=2.0&2.1=3.0&3.2>1000000000&3.2<3000000000|1.2 2.2 3.2"
    single = DistExecutor(dce.NumpyEngine(rels, 0, 1), [rows] * 4).run(query)
    assert DistExecutor(dce.NumpyEngine(rels, 0, 1), [rows] * 4, reorder=False).run(query) == single
    res, nex = _run_world(rels, [query, "0 1|0.1=1.0|0.2 1.2"], world)
    assert res[0] == single
    # whole base relations are bucketed locally (replicated columns): only derived sides move --
    # C3 reordered (R2-sigma(R3), then R1, then R0): one exchange per join; the 2-rel query none
    assert nex == 3
    import agg_truth
    c2 = rels[3][2]
    mask = (c2 > np.uint64(1000000000)) & (c2 < np.uint64(3000000000))
    cnt, nrows, sums = agg_truth.chain4_sums(rels, rows, mask)
    assert res[0][0] == f"{cnt}\n" + "".join(f"{s} " for s in sums) + "\n"
    assert res[0][1] == nrows


def _c5_single_join_cases():
    doc = goldens.load(f"{goldens.GOLDEN_DIR}/c5.json")
    lines, want = [], []
    for c in doc["cases"]:
        body = [l for l in c["input"].splitlines() if l.strip()]
        if len(body) == 1 and c["rc"] == 0 and c["class"] == "T" and body[0].split("|")[1].count("&") == 0 \
                and len(body[0].split("|")[0].split()) == 2:
            lines.append(body[0])
            want.append(c["stdout"])
    return doc, lines, want


def test_agg_plan_single_rank_matches_c5_goldens():
    from qe.dist import DistAggJoin
    doc, lines, want = _c5_single_join_cases()
    rels, _ = goldens.dataset(doc["dataset"])
    ex = DistAggJoin(dce.NumpyEngine(rels, 0, 1), [len(r[0]) for r in rels])
    assert len(lines) >= 4
    for line, w in zip(lines, want):
        assert ex.run(line)[0] == w, line


@pytest.mark.parametrize("world", [2, 3])
def test_agg_plan_heavy_split_matches_c5_goldens(world):
    """the skew path across ranks: heavy keys (sampled) counted per slice and all-reduced, light
    keys bucketed -- same bytes as the reference on every single-join C5 golden"""
    doc, lines, want = _c5_single_join_cases()
    rels, _ = goldens.dataset(doc["dataset"])
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = dce.free_port()
    procs = [ctx.Process(target=dce.agg_worker, args=(r, world, port, rels, lines, q, 1 << 20)) for r in range(world)]
    for p in procs:
        p.start()
    res, _ = q.get(timeout=600)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    for (out, pairs, nheavy), line, w in zip(res, lines, want):
        assert out == w, line
        assert nheavy > 0          # the Zipf head is split, not bucketed
