"""The aggregate push-down checker against the golden vectors G1-G3 (1M rows, real reference
binary) -- CPU only, so the full-size GPU checks stand on a pinned checker."""
import numpy as np

import agg_truth
import goldens
from qe import datagen as dg


def test_chain_truth_matches_headline_goldens():
    doc = goldens.load(goldens.GOLDEN_DIR + "/headline.json")
    cases = {c["input"].strip(): c["stdout"] for c in doc["cases"]}
    rels, _ = goldens.dataset(doc["dataset"])
    N = doc["dataset"]["relations"][0]["rows"]
    c2 = rels[3][2]
    mask = (c2 > np.uint64(1000000000)) & (c2 < np.uint64(3000000000))
    cnt, rows, sums = agg_truth.chain4_sums(rels, N, mask)
    key = "0 1 2 3|0.1=1.0&1.1=2.0&2.1=3.0&3.2>1000000000&3.2<3000000000|1.2 2.2 3.2"
    assert cases[key] == f"{cnt}\n" + "".join(f"{s} " for s in sums) + "\n"
    pairs, s0, s1 = agg_truth.pair_sums(rels[0], rels[1], N)
    assert cases["0 1|0.1=1.0|0.2 1.2"] == f"{s0} {s1} \n"


def test_chain_truth_small_vs_enumeration():
    rels = dg.make_relations(dg.chain_spec(4, 300, 50), 9)
    cnt, rows, sums = agg_truth.chain4_sums(rels, 50)
    # brute force enumeration
    R0, R1, R2, R3 = rels
    tot, s = 0, [0, 0, 0]
    for r1 in range(300):
        a = int(np.sum(R0[1] == R1[0][r1]))
        for r2 in np.nonzero(R2[0] == R1[1][r1])[0]:
            for r3 in np.nonzero(R3[0] == R2[1][r2])[0]:
                tot += a
                s[0] += a * int(R1[2][r1]); s[1] += a * int(R2[2][r2]); s[2] += a * int(R3[2][r3])
    assert rows == tot
    assert sums == [x % (1 << 64) for x in s]


def test_sharded_truth_matches_numpy_small():
    """the torch key-range-sharded checker (used at 1e9 rows on the GPU) against pair_sums on a
    small Zipf case, on the CPU"""
    import torch
    n = 200_000
    rels = dg.make_relations(dg.c5_spec(n), dg.C5_SEED)
    t = [[torch.from_numpy(c.view(np.int64)) for c in r] for r in rels]
    want = agg_truth.pair_sums(rels[0], rels[1], n)
    for shards in (1, 3):
        assert agg_truth.sharded_pair_sums(t[0][1], t[0][2], t[1][0], t[1][2], n, shards) == want
