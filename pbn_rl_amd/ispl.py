"""ISPL network loader: restates the reference's inline ISPL parser.

The reference parses ISPL model files with module-level script code that is
duplicated in train_assa_BQN.py:51-109 and model_tester.py:344-400 (the
1-function variant is train_pbn_assa_BQN.py:51-89).  Its output is what it
passes to ``gym.make("gym-PBN/PBNEnv", N, genes=list(logic_funcs.keys()),
logic_functions=list(logic_funcs.values()))`` (train_assa_BQN.py:121-124,
model_tester.py:409-413): an ordered map gene -> [(python_expr, 1.0), ...].

Rules restated here (line numbers are train_assa_BQN.py):
  * ``Vars:`` block: one gene per line until ``end``; a trailing ``:`` is
    stripped (:62-74).  The reference indexes ``line[0]`` of every line, which
    raises IndexError on the whitespace-only lines the kaban/*.ispl files
    contain; we skip blank lines instead.  The Vars list is informational only:
    the env receives ``logic_funcs.keys()``, i.e. Evolution order (:121-124).
  * ``Evolution:`` block until ``end``, blank lines skipped (:76-86).
  * target gene = text before ``=`` of the first token; ``=false`` guard lines
    are skipped (:88-89).
  * every token ``a=b``: if the last ``=``-part is ``false`` it becomes
    ``( not a )``, otherwise the first part is kept (:91-96).
  * gene ``EGFR`` gets the constant function ``"True"`` (:98-101).
  * expression = tokens[2:] joined by spaces, then ``(``/``)`` padded with
    spaces and ``|``/``&``/``~`` rewritten to ``or``/``and``/``not`` (:103-108).
  * each kept line contributes ``(expr, 1.0)``; duplicates are kept, so a
    repeated function carries weight 2 (:109).
"""
from __future__ import annotations

from collections import OrderedDict
from typing import Iterable, List, Tuple

__all__ = ["parse_ispl", "parse_ispl_file", "IsplNetwork"]

LogicFuncs = "OrderedDict[str, List[Tuple[str, float]]]"


class IsplNetwork:
    """Result of parsing: ``genes`` (Vars order) and ``logic_funcs`` (Evolution order)."""

    def __init__(self, vars_genes: List[str], logic_funcs: "OrderedDict[str, List[Tuple[str, float]]]"):
        self.vars_genes = vars_genes
        self.logic_funcs = logic_funcs

    @property
    def genes(self) -> List[str]:
        # what the reference passes as genes= (train_assa_BQN.py:121-124)
        return list(self.logic_funcs.keys())

    @property
    def logic_functions(self) -> List[List[Tuple[str, float]]]:
        return list(self.logic_funcs.values())


def _rewrite_tokens(tokens: List[str]) -> List[str]:
    out = []
    for tok in tokens:
        parts = tok.split("=")
        if parts[-1] == "false":
            out.append(f"( not {parts[0]} )")
        else:
            out.append(parts[0])
    return out


def _python_syntax(expr: str) -> str:
    expr = expr.replace("(", " ( ")
    expr = expr.replace(")", " ) ")
    expr = expr.replace("|", " or ")
    expr = expr.replace("&", " and ")
    expr = expr.replace("~", " not ")
    return expr


def parse_ispl(lines: Iterable[str]) -> IsplNetwork:
    it = iter(lines)
    vars_genes: List[str] = []
    logic_funcs: "OrderedDict[str, List[Tuple[str, float]]]" = OrderedDict()
    for raw in it:
        line = raw.split()
        if not line:
            continue
        if line[0] == "Vars:":
            for raw2 in it:
                tok = raw2.split()
                if not tok:
                    continue
                if tok[0] == "end":
                    break
                vars_genes.append(tok[0][:-1] if tok[0].endswith(":") else tok[0])
        elif line[0] == "Evolution:":
            for raw2 in it:
                tok = raw2.split()
                if not tok:
                    continue
                if tok[0] == "end":
                    break
                head = tok[0].split("=")
                target = head[0]
                if len(head) > 1 and head[1] == "false":
                    continue
                tok = _rewrite_tokens(tok)
                if target == "EGFR":
                    logic_funcs.setdefault(target, []).append(("True", 1.0))
                    continue
                expr = _python_syntax(" ".join(tok[2:]))
                logic_funcs.setdefault(target, []).append((expr, 1.0))
    return IsplNetwork(vars_genes, logic_funcs)


def parse_ispl_file(path: str) -> IsplNetwork:
    with open(path, "r") as f:
        return parse_ispl(f)
