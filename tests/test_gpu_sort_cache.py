"""The batch's shared base-column sorts (qe_sort_cache, include/qe.h): within one
qe_run_queries_lanes call the first join of a whole base column sorts it once and every later join
on that column reads that sort.  The reference sorts a base relation again for every join
(src/join.c:122-142 allocate_relation + src/join.c:5-94 iterative_sort); the output must not
notice: the C4 goldens (N/100) and the full-size C4 batch byte for byte, with and without the
cache, on 8 lanes and on one."""
import json
import os

import pytest

import goldens
from qe import datagen as dg

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def _c4_small(ctx):
    doc = goldens.load(os.path.join(goldens.GOLDEN_DIR, "c4.json"))
    ctx.drop_relations()
    rels, _ = goldens.dataset(doc["dataset"])
    for cols in rels:
        ctx.load_relation(cols)
    cases = [c for c in doc["cases"] if c["rc"] == 0]
    return "".join(c["input"] for c in cases), "".join(c["stdout"] for c in cases)


def test_c4_goldens_through_the_shared_sorts(ctx, monkeypatch):
    text, want = _c4_small(ctx)
    try:
        h0, b0 = ctx.sort_cache_stats()
        out, rc = ctx.run_lanes(text, 8, plan=True)
        h1, b1 = ctx.sort_cache_stats()
        assert (out, rc) == (want, 0)
        assert b1 - b0 > 0 and h1 - h0 > b1 - b0        # reused more often than built
        out1, rc1 = ctx.run_lanes(text, 1, plan=True)    # one lane (the root ctx builds and reads)
        h2, b2 = ctx.sort_cache_stats()
        assert (out1, rc1) == (want, 0)
        assert h2 - h1 > 0
        monkeypatch.setenv("QE_SORT_CACHE", "0")
        out0, rc0 = ctx.run_lanes(text, 8, plan=True)
        assert (out0, rc0) == (want, 0)
        assert ctx.sort_cache_stats() == (h2, b2)         # off: nothing cached
    finally:
        ctx.drop_relations()


@pytest.mark.slow
def test_c4_full_batch_on_plan_lanes_with_shared_sorts(ctx):
    with open(os.path.join(HERE, "golden", "full", "c4_full.json")) as f:
        doc = json.load(f)
    specs = [dg.RelSpec(r["rows"], [tuple(k) for k in r["kinds"]]) for r in doc["dataset"]["relations"]]
    ctx.drop_relations()
    try:
        for r, sp in enumerate(specs):
            ctx.gen_relation(sp.rows, sp.kinds, seed=doc["dataset"]["seed"], gen_rel=r)
        text = dg.c4_batches([c["input"] for c in doc["cases"]])
        want = "".join(c["stdout"] for c in doc["cases"])
        h0, b0 = ctx.sort_cache_stats()
        out, rc = ctx.run_lanes(text, 8, plan=True)
        h1, b1 = ctx.sort_cache_stats()
        assert (out, rc) == (want, 0)
        assert h1 - h0 > b1 - b0 > 0
    finally:
        ctx.drop_relations()
