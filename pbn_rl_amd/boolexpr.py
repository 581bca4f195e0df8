"""Safe evaluator for the Python-syntax boolean expressions the reference builds.

The reference turns ISPL guards into Python source strings such as
``"( x108208 or x25485 or not x324901 )"`` (train_assa_BQN.py:103-108,
model_tester.py:391-399) and hands them to gym-PBN, which evaluates them as
Python.  Inline networks in the reference use the same syntax directly
(train_pbn_BQN.py:50-88, model_tester.py:71-341).  We never ``eval`` those
strings: this module parses the ``and / or / not / ( ) / True / False / name``
grammar with Python's precedence (not > and > or) and evaluates it over a
variable assignment.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, Dict, List, Sequence, Tuple, Union

import numpy as np

__all__ = ["Expr", "parse", "variables", "evaluate", "ExprError"]


class ExprError(ValueError):
    pass


@dataclass(frozen=True)
class Var:
    name: str


@dataclass(frozen=True)
class Const:
    value: bool


@dataclass(frozen=True)
class Not:
    arg: "Expr"


@dataclass(frozen=True)
class And:
    args: Tuple["Expr", ...]


@dataclass(frozen=True)
class Or:
    args: Tuple["Expr", ...]


Expr = Union[Var, Const, Not, And, Or]

_KEYWORDS = {"and", "or", "not", "(", ")"}


def _tokenize(text: str) -> List[str]:
    spaced = text.replace("(", " ( ").replace(")", " ) ")
    return spaced.split()


def parse(text: str) -> Expr:
    """Parse one expression string; raises ExprError on malformed input."""
    toks = _tokenize(text)
    pos = 0

    def peek() -> str | None:
        return toks[pos] if pos < len(toks) else None

    def take() -> str:
        nonlocal pos
        if pos >= len(toks):
            raise ExprError(f"unexpected end of expression in {text!r}")
        tok = toks[pos]
        pos += 1
        return tok

    def p_or() -> Expr:
        args = [p_and()]
        while peek() == "or":
            take()
            args.append(p_and())
        return args[0] if len(args) == 1 else Or(tuple(args))

    def p_and() -> Expr:
        args = [p_not()]
        while peek() == "and":
            take()
            args.append(p_not())
        return args[0] if len(args) == 1 else And(tuple(args))

    def p_not() -> Expr:
        if peek() == "not":
            take()
            return Not(p_not())
        return p_atom()

    def p_atom() -> Expr:
        tok = take()
        if tok == "(":
            inner = p_or()
            if take() != ")":
                raise ExprError(f"missing ')' in {text!r}")
            return inner
        if tok in _KEYWORDS:
            raise ExprError(f"unexpected {tok!r} in {text!r}")
        if tok == "True":
            return Const(True)
        if tok == "False":
            return Const(False)
        if not (tok[0].isalpha() or tok[0] == "_") or not all(c.isalnum() or c == "_" for c in tok):
            raise ExprError(f"bad identifier {tok!r} in {text!r}")
        return Var(tok)

    tree = p_or()
    if pos != len(toks):
        raise ExprError(f"trailing tokens {toks[pos:]} in {text!r}")
    return tree


def variables(tree: Expr) -> List[str]:
    """Variable names in order of first appearance."""
    out: List[str] = []
    seen = set()

    def walk(node: Expr) -> None:
        if isinstance(node, Var):
            if node.name not in seen:
                seen.add(node.name)
                out.append(node.name)
        elif isinstance(node, Not):
            walk(node.arg)
        elif isinstance(node, (And, Or)):
            for a in node.args:
                walk(a)

    walk(tree)
    return out


def evaluate(tree: Expr, env: Dict[str, bool] | Callable[[str], bool]) -> bool:
    get = env.__getitem__ if isinstance(env, dict) else env
    if isinstance(tree, Var):
        return bool(get(tree.name))
    if isinstance(tree, Const):
        return tree.value
    if isinstance(tree, Not):
        return not evaluate(tree.arg, get)
    if isinstance(tree, And):
        return all(evaluate(a, get) for a in tree.args)
    if isinstance(tree, Or):
        return any(evaluate(a, get) for a in tree.args)
    raise TypeError(tree)


def _evaluate_all(tree: Expr, planes: Dict[str, "np.ndarray"], size: int) -> "np.ndarray":
    if isinstance(tree, Var):
        return planes[tree.name]
    if isinstance(tree, Const):
        return np.full(size, tree.value, dtype=bool)
    if isinstance(tree, Not):
        return ~_evaluate_all(tree.arg, planes, size)
    if isinstance(tree, And):
        out = _evaluate_all(tree.args[0], planes, size).copy()
        for a in tree.args[1:]:
            out &= _evaluate_all(a, planes, size)
        return out
    if isinstance(tree, Or):
        out = _evaluate_all(tree.args[0], planes, size).copy()
        for a in tree.args[1:]:
            out |= _evaluate_all(a, planes, size)
        return out
    raise TypeError(tree)


def compile_truth_table(tree: Expr, inputs: Sequence[str]) -> int:
    """Truth table as an int: bit m is f(x) with inputs[j] = (m >> j) & 1.  All 2^k
    assignments are evaluated at once over numpy bit vectors."""
    k = len(inputs)
    if k > 20:
        raise ExprError(f"arity {k} > 20 is not supported")
    m = np.arange(1 << k, dtype=np.int64)
    planes = {name: ((m >> j) & 1).astype(bool) for j, name in enumerate(inputs)}
    vals = _evaluate_all(tree, planes, 1 << k)
    return int.from_bytes(np.packbits(vals.astype(np.uint8), bitorder="little").tobytes(), "little")
