"""The oracle (oracle/cpu_ref) against the reference's golden vectors -- CPU only.

Pins the C restatement: every golden case produced by the real reference binary
(tests/golden/*.json, oracle/gen_golden.py) must come out byte-identical, exit status
included.  Also pins the generator against SURVEY.md §9.1's check values.
"""
import os
import subprocess

import numpy as np
import pytest

import goldens
from qe import datagen as dg

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CPUREF = os.path.join(ROOT, "oracle", "build", "cpuref")


@pytest.fixture(scope="session", autouse=True)
def _build_cpuref():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "cpuref"], check=True)


def test_generator_check_values():
    # seed 1, N=1e6, r0
    c0 = dg.column(1, 0, 0, 4, ("mod", 1000000))
    c1 = dg.column(1, 0, 1, 3, ("mod", 1000000))
    c2 = dg.column(1, 0, 2, 3, ("hi32",))
    assert c0.tolist() == [413641, 828229, 671478, 794955]
    assert c1.tolist() == [625820, 420461, 115908]
    assert c2.tolist() == [3180582800, 4188313679, 1878341158]
    x = 12345678901234567
    assert int(dg.splitmix64(np.array([x], dtype=np.uint64))[0]) == dg.splitmix64_int(x)


def test_golden_fixtures_present():
    names = {goldens.load(f)["name"] for f in goldens.golden_files()}
    assert {"protocol", "known_answers"} <= names
    n = sum(len(goldens.load(f)["cases"]) for f in goldens.golden_files())
    assert n >= 15


CASES = goldens.all_cases()


@pytest.mark.parametrize("name,idx,ds,case", CASES, ids=[f"{c[0]}-{c[1]}" for c in CASES])
def test_cpuref_matches_reference_golden(name, idx, ds, case):
    rels, paths = goldens.dataset(ds)
    inp = dg.protocol_input(paths, case["input"])
    r = subprocess.run([CPUREF], input=inp.encode(), capture_output=True, timeout=600)
    assert r.stdout.decode("latin-1") == case["stdout"]
    assert r.returncode == case["rc"]
