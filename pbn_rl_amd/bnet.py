"""BoolNet / PyBoolNet ``.bnet`` network loader.

The reference ships bb33 both as ``models/bb33/bb33.ispl`` and as ``models/bb33/bb33.bnet``
(used by ``train_pbn_BQN.py:50-88``'s 33-node network).  A .bnet file has a ``targets, factors``
header and one ``gene, expression`` line per gene; expressions use ``!``, ``&``, ``|``,
parentheses and the constants ``0``/``1``/``true``/``false``.  Every gene gets exactly its one
function (weight 1), i.e. a Boolean network, which is a PBN with one function per node.  The
expressions are rewritten to the Python boolean syntax the reference hands to gym-PBN, so
``Network.from_logic_functions`` compiles them like every other front end; functions of more
than 4 inputs (bb33 has up to 6) are lowered to gates (lowering.py).
"""
from __future__ import annotations

import re
from typing import List, Tuple

from .network import Network

__all__ = ["parse_bnet", "parse_bnet_file"]

_CONST = {"1": "True", "0": "False", "true": "True", "false": "False"}


def _python_expr(expr: str) -> str:
    out = expr.replace("!", " not ").replace("&", " and ").replace("|", " or ")
    return re.sub(r"\b(1|0|true|false)\b", lambda m: _CONST[m.group(1)], out)


def parse_bnet(text: str) -> Tuple[List[str], List[List[Tuple[str, float]]]]:
    """(genes, logic_functions) in the reference's gym-PBN constructor form."""
    genes, funcs = [], []
    for raw in text.splitlines():
        line = raw.split("#", 1)[0].strip()
        if not line or line.replace(" ", "").lower() == "targets,factors":
            continue
        if "," not in line:
            raise ValueError(f"malformed .bnet line {raw!r}")
        target, expr = line.split(",", 1)
        genes.append(target.strip())
        funcs.append([(_python_expr(expr.strip()), 1.0)])
    return genes, funcs


def parse_bnet_file(path: str, name: str = "bnet") -> Network:
    with open(path) as f:
        genes, funcs = parse_bnet(f.read())
    return Network.from_logic_functions(genes, funcs, name=name)
