"""End-to-end parity: every golden vector of the real reference binary (tests/golden/*.json)
through libqe's GPU executor (qe_run_queries) and through the drop-in `queries` binary.
stdout must be byte-identical, stray count lines, NULLs and exit status included."""
import json
import os
import subprocess

import pytest

import goldens
from qe import datagen as dg

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
QUERIES = os.path.join(ROOT, "query-compiler-executor_amd", "build", "queries")

_loaded = {"key": None}


def _load(ctx, ds):
    key = json.dumps(ds, sort_keys=True)
    if _loaded["key"] != key:
        ctx.drop_relations()
        rels, _ = goldens.dataset(ds)
        for cols in rels:
            ctx.load_relation(cols)
        _loaded["key"] = key


CASES = goldens.all_cases()


@pytest.mark.parametrize("name,idx,ds,case", CASES, ids=[f"{c[0]}-{c[1]}" for c in CASES])
def test_gpu_executor_matches_reference_golden(ctx, name, idx, ds, case):
    _load(ctx, ds)
    out, rc = ctx.run(case["input"])
    assert out == case["stdout"]
    assert rc == case["rc"]


def test_gpu_executor_without_dead_list_elimination(ctx, monkeypatch):
    """QE_DLE=0 materialises every intermediate list, as the reference does: same bytes on every
    golden (the default run above has dead-list elimination on)."""
    monkeypatch.setenv("QE_DLE", "0")
    for name, idx, ds, case in CASES:
        _load(ctx, ds)
        out, rc = ctx.run(case["input"])
        assert (out, rc) == (case["stdout"], case["rc"]), (name, idx, case["input"])


@pytest.mark.parametrize("fixture", ["protocol", "known_answers"])
def test_dropin_binary_matches_reference_golden(fixture):
    doc = goldens.load(os.path.join(goldens.GOLDEN_DIR, f"{fixture}.json"))
    rels, paths = goldens.dataset(doc["dataset"])
    for case in doc["cases"]:
        inp = dg.protocol_input(paths, case["input"])
        r = subprocess.run([QUERIES], input=inp.encode(), capture_output=True, timeout=300)
        assert r.stdout.decode("latin-1") == case["stdout"], case["input"]
        assert r.returncode == case["rc"], case["input"]
