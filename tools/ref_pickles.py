"""Read the reference's data pickles WITHOUT unpickling them -> tests/golden/ref_fixtures.json.

    python tools/ref_pickles.py        (build container only: reads /root/reference)

The pickles under /root/reference/data and bns_attractors are never loaded with pickle (nor
with anything that would import or call what a pickle names).  This script walks the opcode
stream with ``pickletools.genops`` -- a disassembler -- and evaluates only a data subset on
its own stack: ints, floats, strings, bytes, tuples, lists, dicts, memo get/put.  A GLOBAL is
kept as an inert ('global', module, name) marker and a REDUCE / BUILD as an inert record of
its operands; nothing named in the file is imported or called.  The two shapes these files
hold are then decoded by hand:
  * attractor lists: list[attractor] of state tuples of 0/1/'*' (model_tester.py:609 maps '*' to 0);
  * model_tester results (model_tester.py:656-658): (save_matrix, data) where save_matrix is a
    float64 numpy array serialised as (_reconstruct, BUILD(shape, dtype, raw bytes)) -- rebuilt
    here with np.frombuffer from the raw bytes -- and data a defaultdict(int) {steps: count}.
"""
import json
import os
import pickletools

import numpy as np

REF = "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden", "ref_fixtures.json")

FILES = {
    "attractors_Bittner-7": "data/attractors_Bittner-7.pkl",
    "attractors_Bittner-28": "data/attractors_Bittner-28.pkl",
    "attractors_pbn10": "bns_attractors/10_3_attractors.pkl",
    "results_pbn_7_4": "data/results/pbn_7_4.pkl",
    "results_pbn_7_6": "data/results/pbn_7_6.pkl",
    "results_pbn_10_6": "data/results/pbn_10_6.pkl",
    "results_pbn_10_26": "data/results/pbn_10_26.pkl",
    "results_pbn_33_3": "data/results/pbn_33_3.pkl",
}

_MARK = object()


def static_eval(data: bytes):
    """Evaluate the data opcodes of a pickle on a private stack; returns the STOP value."""
    stack, memo = [], {}

    def pop_mark():
        i = len(stack) - 1
        while stack[i] is not _MARK:
            i -= 1
        items = stack[i + 1:]
        del stack[i:]
        return items

    for op, arg, _pos in pickletools.genops(data):
        n = op.name
        if n in ("PROTO", "FRAME"):
            continue
        if n == "STOP":
            return stack.pop()
        if n == "MARK":
            stack.append(_MARK)
        elif n in ("BININT", "BININT1", "BININT2", "LONG1", "LONG4", "INT", "LONG",
                   "BINFLOAT", "FLOAT", "SHORT_BINUNICODE", "BINUNICODE", "BINUNICODE8", "UNICODE",
                   "SHORT_BINBYTES", "BINBYTES", "BINBYTES8", "SHORT_BINSTRING", "BINSTRING"):
            stack.append(bytes(arg) if isinstance(arg, (bytes, bytearray)) else arg)
        elif n == "NONE":
            stack.append(None)
        elif n == "NEWTRUE":
            stack.append(True)
        elif n == "NEWFALSE":
            stack.append(False)
        elif n == "EMPTY_LIST":
            stack.append([])
        elif n == "EMPTY_TUPLE":
            stack.append(())
        elif n == "EMPTY_DICT":
            stack.append({})
        elif n == "MEMOIZE":
            memo[len(memo)] = stack[-1]
        elif n in ("BINPUT", "LONG_BINPUT", "PUT"):
            memo[arg] = stack[-1]
        elif n in ("BINGET", "LONG_BINGET", "GET"):
            stack.append(memo[arg])
        elif n == "TUPLE":
            stack.append(tuple(pop_mark()))
        elif n == "TUPLE1":
            stack.append((stack.pop(),))
        elif n == "TUPLE2":
            b, a = stack.pop(), stack.pop()
            stack.append((a, b))
        elif n == "TUPLE3":
            c, b, a = stack.pop(), stack.pop(), stack.pop()
            stack.append((a, b, c))
        elif n == "LIST":
            stack.append(list(pop_mark()))
        elif n == "APPEND":
            v = stack.pop()
            stack[-1].append(v)
        elif n == "APPENDS":
            items = pop_mark()
            stack[-1].extend(items)
        elif n == "DICT":
            items = pop_mark()
            stack.append(dict(zip(items[::2], items[1::2])))
        elif n == "SETITEM":
            v, k = stack.pop(), stack.pop()
            _target(stack[-1])[k] = v
        elif n == "SETITEMS":
            items = pop_mark()
            for k, v in zip(items[::2], items[1::2]):
                _target(stack[-1])[k] = v
        elif n == "STACK_GLOBAL":
            name, module = stack.pop(), stack.pop()
            stack.append(("global", module, name))
        elif n == "GLOBAL":
            module, name = arg.split(" ", 1)
            stack.append(("global", module, name))
        elif n == "REDUCE":   # recorded, never called
            args, fn = stack.pop(), stack.pop()
            stack.append({"reduce": fn, "args": args, "state": None, "items": {}})
        elif n == "BUILD":    # recorded, never applied
            state = stack.pop()
            stack[-1]["state"] = state
        else:
            raise ValueError(f"opcode {n} outside the data subset")
    raise ValueError("no STOP")


def _target(obj):
    return obj["items"] if isinstance(obj, dict) and "reduce" in obj else obj


def decode_ndarray(rec):
    """(_reconstruct(ndarray, (0,), b'b') + BUILD((ver, shape, dtype-record, fortran, raw))) -> array."""
    assert rec["reduce"] == ("global", "numpy.core.multiarray", "_reconstruct"), rec["reduce"]
    _ver, shape, dt, fortran, raw = rec["state"]
    assert dt["reduce"] == ("global", "numpy", "dtype"), dt["reduce"]
    code = dt["args"][0]
    endian = dt["state"][1]
    arr = np.frombuffer(raw, dtype=np.dtype(endian + code if endian in "<>" else code)).reshape(shape)
    return arr.T if fortran else arr


def decode_value(v):
    """0/1/'*' or a numpy scalar record (numpy.core.multiarray.scalar(dtype, raw bytes))."""
    if v == "*" or isinstance(v, int):
        return v
    assert v["reduce"] == ("global", "numpy.core.multiarray", "scalar"), v["reduce"]
    dt, raw = v["args"]
    assert dt["reduce"] == ("global", "numpy", "dtype"), dt["reduce"]
    endian = dt["state"][1]
    code = dt["args"][0]
    return int(np.frombuffer(raw, dtype=np.dtype(endian + code if endian in "<>" else code))[0])


def decode(key, obj):
    if key.startswith("attractors_"):
        return [[[decode_value(v) for v in st] for st in att] for att in obj]
    matrix, hist = obj
    assert hist["reduce"] == ("global", "collections", "defaultdict"), hist["reduce"]
    return {"save_matrix": decode_ndarray(matrix).tolist(),
            "data": {str(k): int(v) for k, v in sorted(hist["items"].items())}}


def main():
    out = {"_source": "tools/ref_pickles.py: static opcode walk of the reference pickles (nothing unpickled)"}
    for key, rel in FILES.items():
        path = os.path.join(REF, rel)
        with open(path, "rb") as f:
            obj = static_eval(f.read())
        out[key] = {"file": rel, "value": decode(key, obj)}
        print(key, json.dumps(out[key]["value"])[:200])
    with open(OUT, "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", OUT)


if __name__ == "__main__":
    main()
