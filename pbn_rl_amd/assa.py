"""ASSA-PBN / MATLAB truth-table network loader.

Restates the text-format reader of train_assa_matlab_BQN.py:72-171 (same layout as
model_tester.py:416-538).  The file is line-oriented:

  two header lines (skipped)                                   :77-81
  n_genes                                                      :83-85
  number of functions of each gene                             :87-90
  number of predictors of each function (all genes, in order)  :92-95
  one line per function: its 2^k truth-table outputs           :102-117
  one line per function: its predictor gene indices            :120-128
  one line per gene: the selection probability of each function  :130-134
  the perturbation rate                                        :136-138

Truth-table column j is the j-th tuple of itertools.product([0, 1], repeat=k) (:112-114), so
predictor 0 is the most significant bit of j.  The reference turns the true columns into a
sympy SOPform expression over the names ``x<index>`` (:144-160) and hands
``genes = [x0 .. x{n-1}]`` with the dict ``{gene index: [(expr, probability), ...]}`` to
``gym.make("gym-PBN/PBNEnv", ...)`` (:162-171).  The perturbation rate is parsed but never
passed on (:136-138, 168-171); ``parse_assa_file`` returns it so a caller can use it.

Here the expression is the disjunction of the true minterms.  It is a different string from
SOPform's minimal form, but it has the same truth table, and that table is all the compiler
(network.py) keeps.
"""
from __future__ import annotations

import itertools
from typing import Dict, List, Tuple

from .network import Network

__all__ = ["AssaNetwork", "parse_assa", "parse_assa_file", "write_assa"]


class AssaNetwork:
    def __init__(self, genes: List[str], logic_functions: Dict[int, List[Tuple[str, float]]], perturbation_rate: float):
        self.genes = genes
        self.logic_functions = logic_functions
        self.perturbation_rate = perturbation_rate

    def network(self, name: str = "assa") -> Network:
        return Network.from_logic_functions(self.genes, self.logic_functions, name=name)


def _sop(names: List[str], outputs: List[float]) -> str:
    k = len(names)
    if k == 0:   # a constant function (no predictors); x0 always exists
        return "x0 or not x0" if outputs[0] else "x0 and not x0"
    minterms = [state for state, out in zip(itertools.product([0, 1], repeat=k), outputs) if out]
    if not minterms:
        return f"{names[0]} and not {names[0]}"           # translate() of 'False' (:62-63)
    if len(minterms) == 1 << k:
        return f"{names[0]} or not {names[0]}"            # translate() of 'True' (:59-60)
    terms = []
    for state in minterms:
        lits = [nm if v else f"not {nm}" for nm, v in zip(names, state)]
        terms.append("(" + " and ".join(lits) + ")")
    return " or ".join(terms)


def parse_assa(text: str) -> AssaNetwork:
    lines = iter(text.splitlines())
    next(lines)
    next(lines)
    n_genes = int(next(lines))
    n_funcs = [int(x) for x in next(lines).split()]
    n_pred = [int(x) for x in next(lines).split()]
    if len(n_funcs) != n_genes or len(n_pred) != sum(n_funcs):
        raise ValueError("function / predictor counts do not match the gene count")
    tables: Dict[int, List[List[float]]] = {}
    fid = 0
    for node in range(n_genes):
        for _ in range(n_funcs[node]):
            vals = [float(x) for x in next(lines).split()]
            if len(vals) != 1 << n_pred[fid]:
                raise ValueError(f"function {fid}: {len(vals)} outputs for {n_pred[fid]} predictors")
            tables.setdefault(node, []).append(vals)
            fid += 1
    preds: Dict[int, List[List[str]]] = {}
    fid = 0
    for node in range(n_genes):
        for _ in range(n_funcs[node]):
            ids = next(lines).split()
            if len(ids) != n_pred[fid]:
                raise ValueError(f"function {fid}: {len(ids)} predictor indices, expected {n_pred[fid]}")
            preds.setdefault(node, []).append([f"x{i}" for i in ids])
            fid += 1
    probas = {node: [float(x) for x in next(lines).split()] for node in range(n_genes)}
    perturbation_rate = float(next(lines))
    logic: Dict[int, List[Tuple[str, float]]] = {}
    for node in range(n_genes):
        if len(probas[node]) != n_funcs[node]:
            raise ValueError(f"gene {node}: {len(probas[node])} probabilities for {n_funcs[node]} functions")
        logic[node] = [(_sop(preds[node][j], tables[node][j]), probas[node][j]) for j in range(n_funcs[node])]
    return AssaNetwork([f"x{i}" for i in range(n_genes)], logic, perturbation_rate)


def parse_assa_file(path: str) -> AssaNetwork:
    with open(path) as f:
        return parse_assa(f.read())


def write_assa(net: Network, perturbation_rate: float = 0.01) -> str:
    """The inverse: ``net`` in the ASSA text layout above (gene i becomes x<i>).  Function
    probabilities are the normalised weights."""
    lines = ["ASSA-PBN model", "written by pbn_rl_amd.assa.write_assa", str(net.n),
             " ".join(str(len(fl)) for fl in net.nodes),
             " ".join(str(f.arity) for fl in net.nodes for f in fl)]
    for fl in net.nodes:
        for f in fl:
            k = f.arity
            outs = []
            for state in itertools.product([0, 1], repeat=k):
                m = sum(v << j for j, v in enumerate(state))   # predictor j = input j of f
                outs.append(str((f.table >> m) & 1))
            lines.append(" ".join(outs) if outs else str(f.table & 1))
    for fl in net.nodes:
        for f in fl:
            lines.append(" ".join(str(g) for g in f.inputs))
    for fl in net.nodes:
        tot = sum(f.weight for f in fl)
        lines.append(" ".join(repr(float(f.weight / tot)) for f in fl))
    lines.append(repr(float(perturbation_rate)))
    return "\n".join(lines) + "\n"
