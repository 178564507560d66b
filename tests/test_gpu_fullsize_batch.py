"""Full-size parity for the two configs whose size the golden vectors cannot reach:

* C4 (BASELINE.json configs[3]): the whole gated batch (874 queries) over the 14 relations of
  qe.datagen.c4_spec(1.0) through the drop-in executor, byte for byte against
  tests/golden/full/c4_full.json -- oracle/cpu_ref's output at full size (oracle/gen_c4_full.py;
  cpu_ref is pinned to the real reference on every golden by tests/test_oracle.py).
* C5 (configs[4]): the Zipf(0.9) 2-relation join at 1e9 rows per side (P ~ 3.8e14 pairs, past the
  materialisation limit and the 46-bit lookback field: the aggregate path at the config's own
  size) against aggregate push-down truth computed by torch on the same device-made columns, one
  key-range shard at a time (no shard holds more than domain/SHARDS counts).
"""
import json
import os

import pytest

import agg_truth
from qe import datagen as dg

pytestmark = [pytest.mark.gpu, pytest.mark.slow]

HERE = os.path.dirname(os.path.abspath(__file__))


def test_c4_full_batch_matches_cpu_ref(ctx):
    with open(os.path.join(HERE, "golden", "full", "c4_full.json")) as f:
        doc = json.load(f)
    specs = [dg.RelSpec(r["rows"], [tuple(k) for k in r["kinds"]]) for r in doc["dataset"]["relations"]]
    assert [(s.rows, s.kinds) for s in specs] == [(s.rows, s.kinds) for s in dg.c4_spec(1.0)]
    ctx.drop_relations()
    try:
        for r, sp in enumerate(specs):
            ctx.gen_relation(sp.rows, sp.kinds, seed=doc["dataset"]["seed"], gen_rel=r)
        queries = [c["input"] for c in doc["cases"]]
        out, rc = ctx.run(dg.c4_batches(queries))        # the reference protocol: batches of 50 + F
        assert rc == 0
        want = "".join(c["stdout"] for c in doc["cases"])
        if out != want:                                   # name the first query that differs
            for c in doc["cases"]:
                got, _ = ctx.run(c["input"])
                assert got == c["stdout"], c["input"]
        assert out == want
    finally:
        ctx.drop_relations()


class _Dev:
    """a libqe device column seen by torch (no copy): __cuda_array_interface__ v2"""

    def __init__(self, ptr, n):
        self.__cuda_array_interface__ = {"shape": (n,), "typestr": "<i8", "data": (ptr, False),
                                         "version": 2, "strides": None}


def test_c5_1e9_against_sharded_aggregate_truth(ctx):
    import torch
    N = dg.C5_ROWS
    ctx.drop_relations()
    try:
        dg.gen_c5(ctx, N)
        out, rc = ctx.run(dg.C5_QUERY)
        assert rc == 0
        pairs_gpu = ctx.last_result_rows()
        ctx.sync()
        cols = {(r, c): torch.as_tensor(_Dev(ctx.column(r, c).d, N), device="cuda") for r in (0, 1) for c in range(3)}
        torch.cuda.synchronize()
        # the query joins r0.c1 = r1.c0 and selects r0.c2, r1.c2
        pairs, s0, s1 = agg_truth.sharded_pair_sums(cols[(0, 1)], cols[(0, 2)], cols[(1, 0)], cols[(1, 2)], N, shards=4)
        del cols
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        assert pairs > (1 << 46)                 # past the merge lookback's 46-bit pair field
        assert pairs_gpu == pairs
        assert out == f"{s0} {s1} \n"
        # the constants bench.py --workload c5 checks its line against
        assert (pairs, out) == (dg.C5_1E9_PAIRS, dg.C5_1E9_STDOUT)
    finally:
        ctx.drop_relations()


def test_c5_1e9_plan_matches_pinned(ctx):
    """the partitioned plan's own path at 1e9 rows (qe_run_queries_dist: the plan's e_join_agg
    bookkeeping, not the faithful executor) against the pinned output"""
    ctx.drop_relations()
    try:
        dg.gen_c5(ctx, dg.C5_ROWS)
        out, rc, refused = ctx.run_dist(dg.C5_QUERY)
        assert rc == 0 and refused == 0
        assert ctx.last_result_rows() == dg.C5_1E9_PAIRS
        assert out == dg.C5_1E9_STDOUT
    finally:
        ctx.drop_relations()
