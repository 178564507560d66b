"""C5 generator on the host (qe.datagen): the Feistel rank->key permutation is a bijection of
[0, D), the Zipf column is deterministic and skewed as specified, and the C5 goldens exist
(the GPU side of the same generator is tests/test_gpu_skew.py)."""
import numpy as np
import pytest

import goldens
from qe import datagen as dg


@pytest.mark.parametrize("domain", [1, 2, 3, 4, 5, 17, 1000, 4096, 20000, 65537, 1 << 20])
def test_feistel_perm_is_a_bijection(domain):
    p = dg.zipf_perm(domain, dg.C5_PERM_SEED)
    assert p.dtype == np.uint64
    assert np.array_equal(np.sort(p), np.arange(domain, dtype=np.uint64))


def test_feistel_perm_depends_on_seed_and_is_pointwise():
    a = dg.zipf_perm(50000, 1)
    b = dg.zipf_perm(50000, 2)
    assert not np.array_equal(a, b)
    x = np.array([0, 7, 49999, 123], dtype=np.uint64)
    assert np.array_equal(dg.feistel_perm(x, 50000, 1), a[x])


def test_zipf_column_shape():
    n, d = 200_000, 20_000
    kind = ("zipf", d, 0.9, dg.C5_PERM_SEED)
    col = dg.column(5, 1, 0, n, kind)
    assert np.array_equal(col, dg.column(5, 1, 0, n, kind))          # deterministic
    assert np.array_equal(col[1000:], dg.column(5, 1, 0, n - 1000, kind, start=1000))
    assert col.max() < d
    # the most frequent key is rank 0's key, with about 1 / H_{d,0.9} of the rows
    h = np.sum(1.0 / np.arange(1, d + 1) ** 0.9)
    vals, cnt = np.unique(col, return_counts=True)
    assert vals[np.argmax(cnt)] == dg.zipf_perm(d, dg.C5_PERM_SEED)[0]
    assert abs(cnt.max() / n - 1.0 / h) < 0.005


def test_c5_spec_and_goldens():
    sp = dg.c5_spec()
    assert [s.rows for s in sp] == [dg.C5_ROWS, dg.C5_ROWS]
    assert sp[0].kinds[1] == sp[1].kinds[0] == ("zipf", dg.C5_ROWS, dg.C5_THETA, dg.C5_PERM_SEED)
    names = {goldens.load(f)["name"] for f in goldens.golden_files()}
    assert {"c5", "c5_theta12"} <= names
    doc = goldens.load(goldens.GOLDEN_DIR + "/c5.json")
    assert doc["cases"][0]["input"] == dg.C5_QUERY and doc["cases"][0]["class"] == "T"
