"""qe_run_queries_parallel: a batch's queries on concurrent lanes (worker contexts on the one GPU,
each its own stream and allocator, the relations shared) must print exactly what the sequential
executor prints -- in input order, cut after the first query where the reference exits."""
import json
import re

import pytest

import goldens

pytestmark = pytest.mark.gpu

WELL_FORMED = re.compile(r"[0-9 ]+\|[0-9.=<>&]+\|[0-9. ]+\n")
_loaded = {"key": None}


def _load(ctx, ds):
    key = json.dumps(ds, sort_keys=True)
    if _loaded["key"] != key:
        ctx.drop_relations()
        rels, _ = goldens.dataset(ds)
        for cols in rels:
            ctx.load_relation(cols)
        _loaded["key"] = key


@pytest.mark.parametrize("workers", [2, 4, 7])
@pytest.mark.parametrize("fixture", ["c4", "fuzz_a", "fuzz_b", "fuzz_c", "protocol"])
def test_parallel_batch_equals_sequential(ctx, fixture, workers):
    doc = goldens.load(f"{goldens.GOLDEN_DIR}/{fixture}.json")
    _load(ctx, doc["dataset"])
    cases = [c for c in doc["cases"] if WELL_FORMED.fullmatch(c["input"]) and c["rc"] == 0]
    text = "".join(c["input"] for c in cases)
    want = "".join(c["stdout"] for c in cases)
    assert ctx.run(text) == (want, 0)
    assert ctx.run_parallel(text, workers) == (want, 0)


def test_parallel_batch_stops_where_the_reference_exits(ctx):
    """K3 (a same-relation same-column join leaves the select without a list: print_sums exits 1)
    in the middle of a batch: the queries before it print, nothing after it does"""
    doc = goldens.load(f"{goldens.GOLDEN_DIR}/fuzz_a.json")
    _load(ctx, doc["dataset"])
    cases = [c for c in doc["cases"] if WELL_FORMED.fullmatch(c["input"]) and c["rc"] == 0][:40]
    bad = "0 0|0.1=0.1|0.2\n"
    text = "".join(c["input"] for c in cases[:25]) + bad + "".join(c["input"] for c in cases[25:])
    want = ctx.run(text)
    assert want[1] == 1
    assert want[0].startswith("".join(c["stdout"] for c in cases[:25]))
    for w in (3, 8):
        assert ctx.run_parallel(text, w) == want
