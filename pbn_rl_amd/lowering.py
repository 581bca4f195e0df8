"""Lowering of wide node functions (more than 4 inputs) to 4-input gates.

The kernels evaluate a node function as a 4-level multiplexer tree over bit-sliced input planes,
so a function record has at most 4 inputs and a 16-bit truth table.  Networks in the reference
go beyond that: bb33 has functions of up to 6 inputs (models/bb33/bb33.ispl, .bnet), and the
inline networks of model_tester.py:98-341 have up to ~20.  Such a function is lowered here into
combinational *gates*. A gate is a function of at most 4 planes, each a node plane or an earlier
gate's output. All of them are evaluated from the same pre-step state s1 as the node functions,
so the synchronous update semantics do not change.

Lowering is a Shannon expansion on the highest input,
    f(x_0..x_{k-1}) = x_{k-1} ? f|_{x_{k-1}=1} : f|_{x_{k-1}=0},
recursing until a cofactor has at most 4 inputs after dropping the inputs it does not depend
on.  Identical sub-functions are shared (hash-consed) across all functions of the network.  The
node's own record becomes the final multiplexer (at most 3 inputs: the split input and two
gate outputs or constants).

A plane reference ("ref") is an int: ``ref < n`` is node ``ref``, ``ref >= n`` is gate ``ref - n``.
Gates are listed in topological order (a gate only reads nodes and earlier gates).
"""
from __future__ import annotations

from typing import Dict, List, Sequence, Tuple

import numpy as np

__all__ = ["Lowering", "lower_network_functions", "MAX_GATES"]

MAX_GATES = 224  # the kernels address planes with one byte: 32 W + gate < 256


def _to_arr(table: int, k: int) -> np.ndarray:
    """Truth table int -> bool array [2]*k, axis a = input k-1-a (C order of the index m)."""
    nbytes = max(1, ((1 << k) + 7) // 8)
    bits = np.unpackbits(np.frombuffer(table.to_bytes(nbytes, "little"), dtype=np.uint8), bitorder="little")
    return bits[: 1 << k].astype(bool).reshape([2] * k) if k else bits[:1].astype(bool).reshape(())


def _to_int(arr: np.ndarray) -> int:
    flat = np.ascontiguousarray(arr).reshape(-1).astype(np.uint8)
    return int.from_bytes(np.packbits(flat, bitorder="little").tobytes(), "little")


def _reduce_refs(inputs: Sequence[int], table: int) -> Tuple[Tuple[int, ...], int]:
    """Drop inputs the function does not depend on and order the rest ascending."""
    k = len(inputs)
    if k == 0:
        return (), table & 1
    A = _to_arr(table, k)
    keep = [j for j in range(k)
            if not np.array_equal(np.take(A, 0, axis=k - 1 - j), np.take(A, 1, axis=k - 1 - j))]
    # drop the others (highest axis first, so the remaining axis numbers stay valid)
    for j in sorted(set(range(k)) - set(keep)):          # ascending j = descending axis
        A = np.take(A, 0, axis=k - 1 - j)
    # A's axes are now the kept inputs, most significant first: axis a = keep[len(keep)-1-a]
    order = sorted(keep, key=lambda j: inputs[j])        # new bit jj = order[jj]
    kk = len(keep)
    if kk == 0:
        return (), int(bool(A))
    pos = {j: kk - 1 - keep.index(j) for j in keep}      # current axis of input j
    A = np.transpose(A, [pos[order[kk - 1 - a]] for a in range(kk)])
    return tuple(inputs[j] for j in order), _to_int(A)


def _cofactor(table: int, k: int, j: int, b: int) -> int:
    """Table over the k-1 inputs left when input j of a k-input table is fixed to b."""
    return _to_int(np.take(_to_arr(table, k), b, axis=k - 1 - j))


class Lowering:
    """Gates shared by all functions of one network with ``n`` nodes."""

    def __init__(self, n: int):
        self.n = n
        self.gates: List[Tuple[Tuple[int, ...], int]] = []      # (input refs, table)
        self._memo: Dict[Tuple[Tuple[int, ...], int], int] = {}

    # a "value" is ("c", bit) for a constant or ("p", ref) for a plane
    def _gate(self, inputs: Tuple[int, ...], table: int):
        if len(inputs) == 1 and table == 0b10:
            return ("p", inputs[0])                               # the input itself
        key = (inputs, table)
        g = self._memo.get(key)
        if g is None:
            g = len(self.gates)
            self.gates.append(key)
            self._memo[key] = g
        return ("p", self.n + g)

    def value(self, inputs: Sequence[int], table: int):
        inputs, table = _reduce_refs(inputs, table)
        k = len(inputs)
        if k == 0:
            return ("c", table & 1)
        if k <= 4:
            return self._gate(inputs, table)
        return self._mux(inputs, table)

    def _mux(self, inputs: Tuple[int, ...], table: int):
        ins, tab = self._mux_function(inputs, table)
        return self._gate(ins, tab) if ins else ("c", tab & 1)

    def _mux_function(self, inputs: Tuple[int, ...], table: int) -> Tuple[Tuple[int, ...], int]:
        """f = v ? f1 : f0 on the last input v, as a function of (v, f0, f1) planes (<= 3 inputs)."""
        k = len(inputs)
        v = inputs[-1]
        f0 = self.value(inputs[:-1], _cofactor(table, k, k - 1, 0))
        f1 = self.value(inputs[:-1], _cofactor(table, k, k - 1, 1))
        planes: List[int] = [v]
        for val in (f0, f1):
            if val[0] == "p" and val[1] not in planes:
                planes.append(val[1])

        def get(val, bits):
            return val[1] if val[0] == "c" else bits[planes.index(val[1])]

        tab = 0
        for m in range(1 << len(planes)):
            bits = [(m >> j) & 1 for j in range(len(planes))]
            out = get(f1, bits) if bits[0] else get(f0, bits)
            if out:
                tab |= 1 << m
        return _reduce_refs(planes, tab)

    def record(self, inputs: Sequence[int], table: int) -> Tuple[Tuple[int, ...], int]:
        """The node-function record (<= 4 input refs, table) computing ``table`` over ``inputs``."""
        inputs, table = _reduce_refs(inputs, table)
        if len(inputs) <= 4:
            return inputs, table
        return self._mux_function(inputs, table)

    def evaluate(self, refs: Sequence[int], table: int, state_bits: Sequence[int]) -> int:
        """Reference evaluation of a record (tests): gates computed on demand from the state."""
        vals: Dict[int, int] = {}

        def plane(r: int) -> int:
            if r < self.n:
                return int(state_bits[r]) & 1
            if r not in vals:
                ins, tab = self.gates[r - self.n]
                m = sum(plane(x) << j for j, x in enumerate(ins))
                vals[r] = (tab >> m) & 1
            return vals[r]

        m = sum(plane(x) << j for j, x in enumerate(refs))
        return (table >> m) & 1


def _op_table(op: str, lits: Sequence[Tuple[int, int]]) -> Tuple[Tuple[int, ...], int]:
    """AND / OR of literals (ref, negated) as (distinct refs ascending, table), reduced."""
    refs = sorted({r for r, _ in lits})
    tab = 0
    for m in range(1 << len(refs)):
        vals = [((m >> refs.index(r)) & 1) ^ neg for r, neg in lits]
        out = all(vals) if op == "and" else any(vals)
        if out:
            tab |= 1 << m
    return _reduce_refs(refs, tab)


class _ExprLowering:
    """Lowers an expression tree (boolexpr) of a wide function.  A subtree over at most 4
    distinct variables becomes one gate (its table by enumeration); a wider AND / OR is
    flattened over nested nodes of the same operator and its operands combined 4 at a time;
    NOT folds into the tables."""

    def __init__(self, low: Lowering, index: Dict[str, int]):
        self.low, self.index = low, index

    def _small(self, tree):
        """("c", bit) | ("l", ref, negated) of a subtree with <= 4 variables."""
        from . import boolexpr as bx
        names = bx.variables(tree)
        refs = [self.index[nm] for nm in names]
        ins, tab = _reduce_refs(refs, bx.compile_truth_table(tree, names))
        if not ins:
            return ("c", tab & 1)
        if len(ins) == 1:
            return ("l", ins[0], 0 if tab == 0b10 else 1)
        return ("l", self.low._gate(ins, tab)[1], 0)

    def literal(self, tree, neg: int = 0):
        from . import boolexpr as bx
        if isinstance(tree, bx.Not):
            return self.literal(tree.arg, neg ^ 1)
        if len(bx.variables(tree)) <= 4:
            v = self._small(tree)
        else:
            op, lits = self.operands(tree)
            if op is None:
                v = lits
            else:
                ins, tab = _op_table(op, lits)
                g = self.low._gate(ins, tab) if ins else ("c", tab & 1)
                v = ("l", g[1], 0) if g[0] == "p" else g
        if not neg:
            return v
        return ("c", v[1] ^ 1) if v[0] == "c" else ("l", v[1], v[2] ^ 1)

    def operands(self, tree):
        """(op, <= 4 literals) of a wide AND / OR, or (None, value) when it folds to one value."""
        from . import boolexpr as bx
        cls = type(tree)
        op = "and" if cls is bx.And else "or"
        absorb = 0 if op == "and" else 1        # the constant that decides the whole node
        flat, stack = [], list(reversed(tree.args))
        while stack:                             # flatten nested nodes of the same operator
            a = stack.pop()
            if type(a) is cls:
                stack.extend(reversed(a.args))
            else:
                flat.append(a)
        lits = []
        for a in flat:
            v = self.literal(a)
            if v[0] == "c":
                if v[1] == absorb:
                    return None, ("c", absorb)
                continue                        # the neutral constant drops out
            lits.append((v[1], v[2]))
        while len(lits) > 4:
            nxt = []
            for c in range(0, len(lits), 4):
                chunk = lits[c:c + 4]
                if len(chunk) == 1:
                    nxt.append(chunk[0])
                    continue
                ins, tab = _op_table(op, chunk)
                g = self.low._gate(ins, tab) if ins else ("c", tab & 1)
                if g[0] == "c":
                    if g[1] == absorb:
                        return None, ("c", absorb)
                    continue
                nxt.append((g[1], 0))
            lits = nxt
        if not lits:
            return None, ("c", 1 - absorb)
        return op, lits

    def record(self, tree) -> Tuple[Tuple[int, ...], int]:
        from . import boolexpr as bx
        neg = 0
        while isinstance(tree, bx.Not):
            tree, neg = tree.arg, neg ^ 1
        if isinstance(tree, (bx.And, bx.Or)) and len(bx.variables(tree)) > 4:
            op, lits = self.operands(tree)
            if op is not None:
                ins, tab = _op_table(op, lits)
                if neg:
                    tab ^= (1 << (1 << len(ins))) - 1
                return ins, tab
            val = lits
        else:
            val = self.literal(tree)
        if neg:
            val = ("c", val[1] ^ 1) if val[0] == "c" else ("l", val[1], val[2] ^ 1)
        if val[0] == "c":
            return (), val[1]
        return (val[1],), (0b01 if val[2] else 0b10)


def lower_network_functions(nodes, genes: Sequence[str] = ()) -> Tuple[Lowering, List[List[Tuple[Tuple[int, ...], int]]]]:
    """Records (<= 4 refs, table) for every function of every node, and the shared gates.

    A function of more than 4 inputs that came from an expression is lowered along its
    expression tree (gates = cut AND / OR nodes); one given only as a table (ASSA files) by
    Shannon expansion."""
    from . import boolexpr as bx
    n = len(nodes)
    low = Lowering(n)
    index = {g: i for i, g in enumerate(genes)}
    recs = []
    for fl in nodes:
        row = []
        for f in fl:
            if f.arity <= 4:
                row.append((tuple(f.inputs), f.table))
                continue
            rec = None
            if f.exprs and index:
                try:
                    rec = _ExprLowering(low, index).record(bx.parse(f.exprs[0]))
                except (KeyError, bx.ExprError):
                    rec = None
            row.append(rec if rec is not None else low.record(f.inputs, f.table))
        recs.append(row)
    return low, recs
