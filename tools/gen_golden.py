"""Generate tests/golden/* fixtures (run in the build container, commit the output).

  python tools/gen_golden.py

1. philox_kat.json   -- rocRAND's philox4x32_10 engine (ten_rounds) outputs for the
                        three Random123 known-answer inputs + 64 seeded random
                        counter/key pairs, produced by oracle/philox_rocrand_kat
                        (built from /opt/rocm/include/rocrand headers).  Pins the
                        oracle's and the kernel's Philox.
2. networks.json     -- per bundled network: node count, function count, canonical
                        truth tables and 16-bit thresholds hash, the Python-eval
                        agreement of every compiled function (reference parser rules,
                        train_assa_BQN.py:51-109), and Bittner-28 fixture self-loop
                        probabilities.
3. steps_<net>.npz   -- oracle step vectors (64 envs x 8 steps, both action modes)
                        for pbn7 / pbn28 / pbn70: inputs and every output, so the
                        CPU suite can detect any drift of the restated semantics.
"""
import hashlib
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)

from oracle import oracle  # noqa: E402
from pbn_rl_amd.attractors import load_attractors  # noqa: E402
from pbn_rl_amd.network import load_network  # noqa: E402
from pbn_rl_amd.spec import EnvSpec  # noqa: E402

GOLDEN = os.path.join(ROOT, "tests", "golden")


def philox_kat():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "kat"], check=True)
    out = subprocess.run([os.path.join(ROOT, "oracle", "philox_rocrand_kat")], check=True,
                         capture_output=True, text=True).stdout
    cases = []
    for line in out.strip().splitlines():
        lhs, rhs = line.split("->")
        v = [int(x, 16) for x in lhs.split()]
        o = [int(x, 16) for x in rhs.split()]
        cases.append({"ctr": v[:4], "key": v[4:6], "out": o})
    with open(os.path.join(GOLDEN, "philox_kat.json"), "w") as f:
        json.dump({"source": "rocRAND philox4x32_10_engine::ten_rounds (ROCm 7.2 headers) via "
                             "oracle/philox_rocrand_kat.cpp; first three = Random123 KAT inputs",
                   "cases": cases}, f, indent=0)
    return len(cases)


def networks():
    from pbn_rl_amd import boolexpr

    rec = {}
    for name in ["pbn7", "pbn10", "pbn28", "pbn70"]:
        net = load_network(name)
        # every compiled function agrees with a direct evaluation of its source expressions
        agree = 0
        rng = np.random.default_rng(0)
        for i, fl in enumerate(net.nodes):
            for f in fl:
                for expr in f.exprs:
                    tree = boolexpr.parse(expr)
                    for _ in range(16):
                        bits = rng.integers(0, 2, size=net.n)
                        env = {g: bool(bits[k]) for k, g in enumerate(net.genes)}
                        assert boolexpr.evaluate(tree, env) == bool(f(bits))
                        agree += 1
        arr = net.descriptor_arrays(16)
        keys = ["func_arity", "func_inputs", "func_table", "func_threshold", "node_func_start"]   # = tests/test_network.py
        h = hashlib.sha256(b"".join(arr[k].tobytes() for k in keys)).hexdigest()
        rec[name] = {"n_nodes": net.n, "n_funcs": int(arr["func_arity"].shape[0]),
                     "descriptor_sha256": h, "checked_evaluations": agree,
                     "attractors": len(load_attractors(name))}
    net = load_network("pbn28")
    rec["pbn28"]["fixture_self_loop"] = [
        round(net.self_loop_probability(list(att[0]), 16), 6) for att in load_attractors("pbn28")]
    with open(os.path.join(GOLDEN, "networks.json"), "w") as f:
        json.dump(rec, f, indent=1)
    return rec


def steps():
    for name in ["pbn7", "pbn28", "pbn70"]:
        spec = EnvSpec(load_network(name), load_attractors(name), perturbation=0.05)
        n, seed, off = 64, 987654321, 32
        W = spec.words
        rng = np.random.default_rng(11)
        st, tg, t = oracle.reset(spec, seed, 0, off, n)
        data = {"reset_state": st.copy(), "reset_target": tg.copy(), "reset_t": t.copy()}
        for k in range(8):
            mode = 3 if k % 2 == 0 else 1
            flip = np.zeros((W, n), dtype=np.uint32)
            if mode == 1:
                flip = rng.integers(0, 2 ** 32, size=(W, n), dtype=np.uint64).astype(np.uint32)
                flip &= np.uint32(0x01010101)
            out = oracle.step(spec, seed, k + 1, off, st, flip, tg, t, mode)
            data[f"in_state_{k}"] = st
            data[f"in_flip_{k}"] = flip
            data[f"in_target_{k}"] = tg
            data[f"in_t_{k}"] = t
            for key in ("state_out", "final_state", "reward", "flags", "target", "t", "flipmask"):
                data[f"out_{key}_{k}"] = out[key]
            st, tg, t = out["state_out"], out["target"], out["t"]
        np.savez_compressed(os.path.join(GOLDEN, f"steps_{name}.npz"), seed=seed, env_offset=off,
                            perturbation=0.05, **data)


if __name__ == "__main__":
    os.makedirs(GOLDEN, exist_ok=True)
    print("philox cases", philox_kat())
    print(json.dumps(networks())[:300])
    steps()
    print("steps fixtures written")
