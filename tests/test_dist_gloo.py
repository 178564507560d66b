"""The C5 skew plan (qe.dist.DistAggJoin) on CPU: world_size 1, 2 and 3 under torch.distributed
gloo with a numpy engine, against the reference's C5 goldens.  (The relational plan, host C, is
tested the same way by tests/test_plan_gloo.py.)"""
import pytest
import torch.multiprocessing as mp

import dist_cpu_engine as dce
import goldens


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
