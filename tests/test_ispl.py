"""ISPL parser (restating train_assa_BQN.py:51-109) and the safe expression evaluator."""
import ast
import json
import os

import numpy as np
import pytest

from pbn_rl_amd import boolexpr
from pbn_rl_amd.ispl import parse_ispl
from pbn_rl_amd.network import NETWORK_DIR, Network

SAMPLE = """Agent M
\tVars:
\t\t
\t\tA: boolean;
\t\t
\t\tB: boolean;
\t\tEGFR: boolean;
\tend Vars
\tEvolution:
\t\t
\t\tA=true if (B |  ~ A)=true;
\t\tA=false if (B |  ~ A)=false;
\t\tA=true if (B |  ~ A)=true;
\t\tB=true if (( A &  B) |  ~ EGFR)=true;
\t\tEGFR=true if (A)=true;
\tend Evolution
end Agent
"""


def test_parser_rules():
    net = parse_ispl(SAMPLE.splitlines(True))
    assert net.vars_genes == ["A", "B", "EGFR"]          # blank Vars lines skipped
    assert net.genes == ["A", "B", "EGFR"]               # Evolution order (train_assa_BQN.py:121-124)
    lf = net.logic_functions
    assert len(lf[0]) == 2 and lf[0][0] == lf[0][1]       # duplicates kept (weight 2), =false lines skipped
    assert lf[0][0][1] == 1.0
    assert lf[0][0][0].split() == ["(", "B", "or", "not", "A", ")"]
    assert lf[2] == [("True", 1.0)]                       # EGFR special case (:98-101)


def _py_eval(expr, env):
    """Evaluate the Python-syntax expression through the ast module (no exec)."""
    def ev(n):
        if isinstance(n, ast.Expression):
            return ev(n.body)
        if isinstance(n, ast.BoolOp):
            vals = [ev(v) for v in n.values]
            return all(vals) if isinstance(n.op, ast.And) else any(vals)
        if isinstance(n, ast.UnaryOp) and isinstance(n.op, ast.Not):
            return not ev(n.operand)
        if isinstance(n, ast.Name):
            return env[n.id]
        if isinstance(n, ast.Constant):
            return bool(n.value)
        raise TypeError(n)
    return ev(ast.parse(expr.strip(" \t"), mode="eval"))  # eval() strips leading blanks too


@pytest.mark.parametrize("name", ["pbn7", "pbn10", "pbn28", "pbn70"])
def test_compiled_functions_match_python_semantics(name):
    with open(os.path.join(NETWORK_DIR, f"{name}.json")) as f:
        obj = json.load(f)
    net = Network.from_json(obj)
    rng = np.random.default_rng(1)
    for i, fl in enumerate(net.nodes):
        for fn in fl:
            for expr in fn.exprs:
                for _ in range(8):
                    bits = rng.integers(0, 2, size=net.n)
                    env = {g: bool(bits[k]) for k, g in enumerate(net.genes)}
                    want = _py_eval(expr, env)
                    assert boolexpr.evaluate(boolexpr.parse(expr), env) == want
                    assert fn(bits) == int(want)


@pytest.mark.parametrize("name", ["pbn7", "pbn10", "pbn28", "pbn70"])
def test_bundled_json_matches_reference_ispl(name, reference_dir):
    net = Network.from_ispl(os.path.join(reference_dir, "kaban", f"{name}.ispl"), name=name)
    with open(os.path.join(NETWORK_DIR, f"{name}.json")) as f:
        obj = json.load(f)
    assert net.genes == obj["genes"]
    assert [[list(x) for x in fl] for fl in net.logic_functions] == obj["logic_functions"]


def test_expression_errors():
    for bad in ["( a or", "a b", "and a", "a or ( )", "1abc"]:
        with pytest.raises(boolexpr.ExprError):
            boolexpr.parse(bad)
    assert boolexpr.evaluate(boolexpr.parse("not not a and ( b or False )"), {"a": True, "b": True})
