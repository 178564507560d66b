"""End-to-end parity: every golden vector of the real reference binary (tests/golden/*.json)
through libqe's GPU executor (qe_run_queries) and through the drop-in `queries` binary.
stdout must be byte-identical, stray count lines, NULLs and exit status included."""
import json
import os
import re
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


WELL_FORMED = re.compile(r"[0-9 ]+\|[0-9.=<>&]+\|[0-9. ]+\n")


def _binary(paths, queries, env=None):
    r = subprocess.run([QUERIES], input=dg.protocol_input(paths, queries).encode(), capture_output=True, timeout=600,
                       env=dict(os.environ, **(env or {})))
    return r.stdout.decode("latin-1"), r.returncode


MODES = {
    "default": {},                                        # the plan on 8 lanes, faithful fallback
    "nocache": {"QE_SORT_CACHE": "0"},                    # ... without the batch's shared base-column sorts
    "faithful": {"QE_PLAN": "0", "QE_WORKERS": "1"},      # the reference's state machine, one lane
    "plan1": {"QE_WORKERS": "1"},                         # the plan, one lane
    "ranks1": {"QE_GPUS": "1"},                           # rank launcher: fork, RCCL id over a pipe
    "lanes4": {"QE_PLAN": "0", "QE_WORKERS": "4"},        # the faithful executor on four lanes
    "agg0": {"QE_PLAN": "0", "QE_AGG_MIN": "0"},          # faithful, aggregate last join at any size
    "local3": {"QE_LOCAL_RANKS": "3"},                    # three in-process ranks: real exchanges
    # the plan's multi-rank aggregate join (e_join_agg: heavy keys by row slice, light hash
    # buckets) at golden sizes, which stay below its default minimum (QE_AGG_MIN, read once per
    # process: set before the binary starts)
    "local2agg0": {"QE_LOCAL_RANKS": "2", "QE_AGG_MIN": "0"},
    "local3agg0": {"QE_LOCAL_RANKS": "3", "QE_AGG_MIN": "0"},
    "local8agg0": {"QE_LOCAL_RANKS": "8", "QE_AGG_MIN": "0"},
}


@pytest.mark.parametrize("mode", list(MODES))
@pytest.mark.parametrize("fixture", [os.path.basename(f)[:-5] for f in goldens.golden_files()])
def test_dropin_binary_matches_reference_golden(fixture, mode):
    """every golden through build/queries (mmap'd relation files, the reference's stdin protocol).
    Well-formed single-line queries that exit 0 run as one batch per fixture -- every line fills
    all three of the parser's scan buffers, so no line sees another's leftovers -- and the batch's
    stdout is the concatenation of theirs; every other case (malformed lines, exit(1), multi-line
    inputs) runs on its own."""
    env = MODES[mode]
    doc = goldens.load(os.path.join(goldens.GOLDEN_DIR, f"{fixture}.json"))
    rels, paths = goldens.dataset(doc["dataset"])
    batch = [c for c in doc["cases"] if c["rc"] == 0 and WELL_FORMED.fullmatch(c["input"])]
    alone = [c for c in doc["cases"] if c not in batch]
    if batch:
        out, rc = _binary(paths, "".join(c["input"] for c in batch), env)
        want = "".join(c["stdout"] for c in batch)
        if out != want:
            for c in batch:
                assert _binary(paths, c["input"], env) == (c["stdout"], 0), c["input"]
        assert (out, rc) == (want, 0)
    for case in alone:
        assert _binary(paths, case["input"], env) == (case["stdout"], case["rc"]), case["input"]


@pytest.mark.parametrize("cut", [0, 8, 16, 40, -8])
def test_dropin_binary_rejects_a_truncated_relation_file(tmp_path, cut):
    """a relation file shorter than its header says (cut bytes kept; -8: one value short) ends the
    run with a message and exit status 1 -- not a SIGBUS (the reference check()s open / fstat /
    mmap, src/utilities.c:136-146)"""
    rels = dg.make_relations(dg.chain_spec(2, 1000), 1)
    paths = dg.write_dataset(str(tmp_path), rels)
    data = open(paths[1], "rb").read()
    open(paths[1], "wb").write(data[:cut] if cut >= 0 else data[:cut])
    r = subprocess.run([QUERIES], input=dg.protocol_input(paths, "0 1|0.1=1.0|0.2 1.2\n").encode(),
                       capture_output=True, timeout=120)
    assert r.returncode == 1, (r.returncode, r.stderr)
    assert r.stdout == b""
    assert b"[ERROR]" in r.stderr
