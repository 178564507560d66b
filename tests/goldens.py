"""Golden-vector helpers shared by the oracle, host and GPU parity tests.

Golden fixtures (tests/golden/*.json) hold generator parameters, query text and the exact stdout
bytes + exit status of the real reference binary (oracle/gen_golden.py).
The relation files are regenerated here, bit-exact, from qe.datagen.
"""
from __future__ import annotations

import glob
import json
import os
import tempfile

from qe import datagen as dg

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN_DIR = os.path.join(HERE, "golden")
_CACHE: dict = {}


def golden_files(include_headline: bool = True) -> list[str]:
    fs = sorted(glob.glob(os.path.join(GOLDEN_DIR, "*.json")))
    if not include_headline:
        fs = [f for f in fs if not os.path.basename(f).startswith("headline")]
    return fs


def load(path: str) -> dict:
    with open(path) as f:
        return json.load(f)


def dataset(ds: dict):
    """(relations as numpy columns, file paths) for a fixture's dataset; cached per process."""
    key = json.dumps(ds, sort_keys=True)
    if key not in _CACHE:
        specs = [dg.RelSpec(r["rows"], [tuple(k) for k in r["kinds"]]) for r in ds["relations"]]
        rels = dg.make_relations(specs, ds["seed"])
        d = tempfile.mkdtemp(prefix="qe_golden_")
        paths = dg.write_dataset(d, rels)
        _CACHE[key] = (rels, paths)
    return _CACHE[key]


def all_cases(include_headline: bool = True):
    """[(fixture name, case index, dataset dict, case dict)]"""
    out = []
    for f in golden_files(include_headline):
        doc = load(f)
        for i, c in enumerate(doc["cases"]):
            out.append((doc["name"], i, doc["dataset"], c))
    return out
