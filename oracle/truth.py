"""Relational-truth evaluator (diagnostic only).  TEST INFRASTRUCTURE ONLY.

Evaluates a query line with textbook semantics -- filters, then equi-joins (the reference
ignores the join operator, src/join.c:325-392, so every join is an equality here too) -- and
returns the stdout line the query *should* print.  Used to label golden vectors T (reference
== relational truth) or W (deterministic but wrong); W goldens still bind the build
(SURVEY.md §8(c) item 2).  Not a parity oracle: the reference binary (oracle/_ref) and
oracle/cpu_ref are.
"""
from __future__ import annotations

import re

import numpy as np
import pandas as pd

M64 = (1 << 64) - 1


def parse(line: str):
    rels_s, preds_s, sel_s = line.strip().split("|")
    rels = [int(x) for x in rels_s.split(" ")]
    joins, filters = [], []
    for p in preds_s.split("&"):
        m = re.fullmatch(r"(\d+)\.(\d+)([=<>])(\d+)\.(\d+)", p)
        if m:
            a, b, op, c, d = m.groups()
            joins.append((int(a), int(b), int(c), int(d)))
            continue
        m = re.fullmatch(r"(\d+)\.(\d+)([=<>])(\d+)", p)
        a, b, op, c = m.groups()
        filters.append((int(a), int(b), op, int(c) & 0xFFFFFFFF))
    sels = [tuple(int(v) for v in s.split(".")) for s in sel_s.split(" ")]
    return rels, joins, filters, sels


def evaluate(line: str, relations: list[list[np.ndarray]]) -> str:
    rels, joins, filters, sels = parse(line)
    nb = len(rels)
    cand = {}
    for b in range(nb):
        cand[b] = np.arange(len(relations[rels[b]][0]), dtype=np.int64)
    for (b, c, op, v) in filters:
        col = relations[rels[b]][c][cand[b]]
        v64 = np.uint64(v)
        keep = col == v64 if op == "=" else (col > v64 if op == ">" else col < v64)
        cand[b] = cand[b][keep]
    # components: each is a DataFrame with one int64 rowid column per binding
    comp = {b: pd.DataFrame({b: cand[b]}) for b in range(nb)}
    owner = {b: b for b in range(nb)}

    def keycol(df, b, c):
        return relations[rels[b]][c][df[b].to_numpy()]

    for (b1, c1, b2, c2) in joins:
        o1, o2 = owner[b1], owner[b2]
        if o1 == o2:
            df = comp[o1]
            keep = keycol(df, b1, c1) == keycol(df, b2, c2)
            comp[o1] = df[keep].reset_index(drop=True)
            continue
        d1, d2 = comp[o1], comp[o2]
        k1 = d1.assign(__k=keycol(d1, b1, c1))
        k2 = d2.assign(__k=keycol(d2, b2, c2))
        merged = k1.merge(k2, on="__k", how="inner").drop(columns="__k")
        comp[o1] = merged
        del comp[o2]
        for b in range(nb):
            if owner[b] == o2:
                owner[b] = o1
    # a disconnected query is a cross product of its components
    roots = sorted(set(owner.values()))
    sizes = {r: len(comp[r]) for r in roots}
    total = 1
    for r in roots:
        total *= sizes[r]
    out = []
    for (b, c) in sels:
        r = owner[b]
        if total == 0:
            out.append("NULL ")
            continue
        mult = total // sizes[r]
        vals = relations[rels[b]][c][comp[r][b].to_numpy()]
        s = int(np.sum(vals, dtype=np.uint64)) if len(vals) else 0
        out.append(f"{(s * mult) & M64} ")
    return "".join(out) + "\n"


def truth_sums(line: str, relations) -> str:
    return evaluate(line, relations)
