"""ctypes wrapper around oracle/libpbn_oracle.so (the C restatement).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, as the checker.  Host numpy arrays in the same
SoA layout as the device buffers of include/pbn_env.h.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# PBN_ORACLE_LIB selects another build of the same source (the ASan one, tests/test_oracle_asan.py)
LIB_PATH = os.environ.get("PBN_ORACLE_LIB") or os.path.join(HERE, "libpbn_oracle.so")
_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE, "all"], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        vp, u64, i64, u32, i32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int64, ctypes.c_uint32, ctypes.c_int
        L.oracle_step.argtypes = [vp, u64, u64, u64, i64, u32, vp, vp, vp, vp, vp, vp, vp, vp, i32]
        L.oracle_step.restype = i32
        L.oracle_step_ex.argtypes = [vp, u64, u64, u64, i64, u32, vp, vp, vp, vp, vp, vp, vp, vp, vp, i32]
        L.oracle_step_ex.restype = i32
        L.oracle_reset.argtypes = [vp, u64, u64, u64, i64, vp, vp, vp]
        L.oracle_reset.restype = i32
        L.oracle_philox4x32_10.argtypes = [vp, vp, vp]
        L.oracle_philox4x32_10.restype = None
        L.oracle_philox4x32_r.argtypes = [vp, vp, vp, i32]
        L.oracle_philox4x32_r.restype = None
        _lib = L
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data


def philox(ctr, key, rounds: int = 10):
    """Philox4x32-R of the C oracle (10 = rocRAND's philox4x32_10; the streams draw R = 7)."""
    c = np.ascontiguousarray(ctr, dtype=np.uint32)
    k = np.ascontiguousarray(key, dtype=np.uint32)
    out = np.zeros(4, dtype=np.uint32)
    if rounds == 10:
        lib().oracle_philox4x32_10(_p(c), _p(k), _p(out))
    else:
        lib().oracle_philox4x32_r(_p(c), _p(k), _p(out), rounds)
    return out


def reset(spec, seed: int, step: int, env_offset: int, n: int):
    W = spec.words
    state = np.zeros((W, n), dtype=np.uint32)
    target = np.zeros(n, dtype=np.uint8)
    t = np.zeros(n, dtype=np.uint8)
    rc = lib().oracle_reset(ctypes.addressof(spec.desc), seed, step, env_offset, n,
                            _p(state), _p(target), _p(t))
    assert rc == 0
    return state, target, t


def step(spec, seed: int, step: int, env_offset: int, state, flipmask, target, t, mode: int,
         want_final: bool = True, n_threads: int = 0):
    """Returns dict of outputs; target/t are returned updated (inputs are not modified).
    ``updates``: the synchronous updates applied per env (the settle length under the settle law)."""
    W, n = state.shape
    state = np.ascontiguousarray(state, dtype=np.uint32)
    flip = np.ascontiguousarray(flipmask, dtype=np.uint32).copy()
    tgt = np.ascontiguousarray(target, dtype=np.uint8).copy()
    tt = np.ascontiguousarray(t, dtype=np.uint8).copy()
    out = np.zeros((W, n), dtype=np.uint32)
    final = np.zeros((W, n), dtype=np.uint32) if want_final else None
    reward = np.zeros(n, dtype=np.float32)
    flags = np.zeros(n, dtype=np.uint8)
    updates = np.zeros(n, dtype=np.uint16)
    rc = lib().oracle_step_ex(ctypes.addressof(spec.desc), seed, step, env_offset, n, mode,
                              _p(state), _p(flip), _p(tgt), _p(tt), _p(out), _p(final), _p(reward),
                              _p(flags), _p(updates), n_threads)
    if rc != 0:
        raise ValueError(f"oracle_step failed ({rc})")
    return {"state_out": out, "final_state": final, "reward": reward, "flags": flags,
            "target": tgt, "t": tt, "flipmask": flip, "updates": updates}
