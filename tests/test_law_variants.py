"""The step-law variants scored against the reference's trained-agent evaluations
(tests/law_variants.py, profiles/r04_law_variants.json; DESIGN.md "Parity status").

The committed table is the documented negative result of VERDICT r03's next item 2: no variant
of the law (one update / settle to any attractor / settle to the target; perturbation in the
settle updates or not; p = 0 or 0.01; distinct or raw action flips; pbn10 in either gene order)
reproduces data/results/pbn_10_6.pkl or pbn_7_4.pkl.  These tests re-derive one row exactly and
check the table's conclusion.
"""
import json
import os

import numpy as np
import pytest

from . import law_variants as lv

TABLE = os.path.join(lv.ROOT, "profiles", "r04_law_variants.json")


def rows():
    with open(TABLE) as f:
        return json.load(f)["rows"]


def test_no_variant_reproduces_the_recorded_evaluations():
    """A variant matches a fixture when its expected failures are below one (the reference
    recorded none) and its expected one-step runs lie within 3 standard deviations of the
    recorded count (binomial over the off-diagonal runs)."""
    for r in rows():
        n = r["recorded"]["runs"]
        q = r["e_one"] / n
        sd = np.sqrt(n * q * (1 - q)) + 1e-9
        matches = r["e_fail"] < 1.0 and abs(r["e_one"] - r["recorded"]["one"]) < 3 * sd
        assert not matches, r


def test_best_pbn10_variant_is_settle_to_target():
    """In the agent's gene order the best-scoring law for pbn10 runs each step to the target
    attractor (0 expected failures, as recorded) but over-predicts the one-step runs."""
    best = max((r for r in rows() if r["fixture"] == "pbn_10_6/lex"), key=lambda r: r["ll_hist"])
    assert best["law"] == "target" and best["p"] == 0.01 and best["pert_in_settle"]
    assert best["e_fail"] < 0.5 and best["e_one"] > best["recorded"]["one"] + 30


@pytest.mark.parametrize("law_kind", ["settle", "target"])
def test_table_row_reproduces(law_kind):
    case = [c for c in lv.fixture_cases() if c[0] == "pbn_10_6/lex"][0]
    name, net, atts, q_fn, data, matrix = case
    res = lv.protocol(net, atts, q_fn, law_kind=law_kind, pert=True, p=0.01, mode="or")
    got = lv.scores(res, data, matrix)
    want = [r for r in rows() if r["fixture"] == name and r["law"] == law_kind and r["p"] == 0.01
            and r["pert_in_settle"] and r["actions"] == "or"][0]
    for k in ("ll_hist", "ll_matrix", "e_fail", "e_one"):
        assert abs(got[k] - want[k]) < 1e-6 * max(1.0, abs(want[k])), k
