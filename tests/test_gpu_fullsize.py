"""Full-size parity (BASELINE.json configs at 100 M rows/relation) on the GPU executor, checked
against the aggregate push-down truth (tests/agg_truth.py, itself pinned to the reference's
golden vectors G1-G3 by tests/test_agg_truth.py).  Both configs are in the class where the
reference equals relational truth."""
import numpy as np
import pytest

import agg_truth
from qe import datagen as dg

pytestmark = [pytest.mark.gpu, pytest.mark.slow]

N = 100_000_000
C3 = "0 1 2 3|0.1=1.0&1.1=2.0&2.1=3.0&3.2>1000000000&3.2<3000000000|1.2 2.2 3.2\n"
C2 = "0 1|0.1=1.0|0.2 1.2\n"


@pytest.fixture(scope="module")
def full(ctx):
    rels = dg.make_relations(dg.chain_spec(4, N), 1)
    ctx.drop_relations()
    kinds = [("mod", N), ("mod", N), ("hi32",)]
    for r in range(4):
        ctx.gen_relation(N, kinds, seed=1, gen_rel=r)   # generated on the GPU ...
    # ... and equal to the host generator (whole-column checksums)
    for r in range(4):
        for c in range(3):
            assert ctx.checksum(ctx.column(r, c), None) == int(np.sum(rels[r][c], dtype=np.uint64))
    yield rels
    ctx.drop_relations()


def test_c3_chain_100m(ctx, full):
    out, rc = ctx.run(C3)
    c2 = full[3][2]
    mask = (c2 > np.uint64(1000000000)) & (c2 < np.uint64(3000000000))
    cnt, rows, sums = agg_truth.chain4_sums(full, N, mask)
    assert rc == 0
    assert out == f"{cnt}\n" + "".join(f"{s} " for s in sums) + "\n"
    assert ctx.last_result_rows() == rows


def test_c2_pair_100m(ctx, full):
    out, rc = ctx.run(C2)
    pairs, s0, s1 = agg_truth.pair_sums(full[0], full[1], N)
    assert rc == 0
    assert out == f"{s0} {s1} \n"
    assert ctx.last_result_rows() == pairs


@pytest.mark.parametrize("side_stream", ["0", "1"])
def test_c3_planned_with_and_without_the_side_stream(ctx, full, side_stream, monkeypatch):
    """the partitioned plan on C3 with each join's two sorts on one stream, and (QE_SIDE_STREAM=1)
    with one side's sort on the ctx's side stream concurrently with the other's (SideFork: the side
    stream's own lookback words and scratch, frees held until the streams meet): the same bytes as
    the aggregate truth, three times in a row (the held blocks recycled between queries)"""
    monkeypatch.setenv("QE_SIDE_STREAM", side_stream)
    c2 = full[3][2]
    mask = (c2 > np.uint64(1000000000)) & (c2 < np.uint64(3000000000))
    cnt, rows, sums = agg_truth.chain4_sums(full, N, mask)
    want = f"{cnt}\n" + "".join(f"{s} " for s in sums) + "\n"
    for _ in range(3):
        out, rc, refused = ctx.run_dist(C3)
        assert (out, rc, refused) == (want, 0, 0)
        assert ctx.last_result_rows() == rows
