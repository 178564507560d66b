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
    res, nex = _run_world(rels, [query, "0 1|0.1=1.0|0.2 1.2"], world)
    assert res[0] == single
    assert nex == 3 * 2 + 1 * 2   # one exchange per join side
    import agg_truth
    c2 = rels[3][2]
    mask = (c2 > np.uint64(1000000000)) & (c2 < np.uint64(3000000000))
    cnt, nrows, sums = agg_truth.chain4_sums(rels, rows, mask)
    assert res[0][0] == f"{cnt}\n" + "".join(f"{s} " for s in sums) + "\n"
    assert res[0][1] == nrows
