"""EnvSpec: everything that defines one PBN environment, as a C descriptor.

An EnvSpec bundles the compiled network (network.py), the attractor set that
drives reset()/reward (attractors.py), the perturbation probability, the
selection-probability resolution, the horizon and the reward constants.  It
produces the ``pbn_net_desc`` struct of include/pbn_env.h (ctypes), which both
libpbn_env.so and the test oracle consume.

Reward (frozen; gym_PBN's own reward is unavailable -- SURVEY.md section 8(a) A7):
    r = success_reward * terminated
        - wrong_attractor_cost * [s' in an attractor other than the target]
        - action_cost * (number of intervened nodes)
        - step_cost
evaluated in float64 and stored as a float32 table indexed by
(terminated, wrong, popcount(flipmask)); the device only looks it up.
Defaults: success 5, wrong attractor 2, action 1, step 0 (constructor kwargs).
"""
from __future__ import annotations

import ctypes
from typing import Optional, Sequence

import numpy as np

from .attractors import Attractors, clean_state
from .network import Network, perturbation_cdf

__all__ = ["EnvSpec", "PbnNetDesc", "NO_TARGET"]

NO_TARGET = 0xFF
MAX_ATTRACTORS = 254
MAX_SETTLE = 4096


class PbnNetDesc(ctypes.Structure):
    _fields_ = [
        ("n_nodes", ctypes.c_int32),
        ("n_funcs", ctypes.c_int32),
        ("prob_bits", ctypes.c_int32),
        ("horizon", ctypes.c_int32),
        ("node_func_start", ctypes.c_void_p),
        ("func_arity", ctypes.c_void_p),
        ("func_inputs", ctypes.c_void_p),
        ("func_table", ctypes.c_void_p),
        ("func_threshold", ctypes.c_void_p),
        ("perturb_cdf", ctypes.c_void_p),
        ("n_attractors", ctypes.c_int32),
        ("n_attractor_states", ctypes.c_int32),
        ("attractor_start", ctypes.c_void_p),
        ("attractor_states", ctypes.c_void_p),
        ("reward_table", ctypes.c_void_p),
        ("n_gates", ctypes.c_int32),
        ("gate_arity", ctypes.c_void_p),
        ("gate_inputs", ctypes.c_void_p),
        ("gate_table", ctypes.c_void_p),
        ("settle_max", ctypes.c_int32),
    ]


def _ptr(a: np.ndarray) -> int:
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data


class EnvSpec:
    def __init__(self, network: Network, attractors: Optional[Attractors] = None, *,
                 perturbation: float = 0.01, prob_bits: int = 16, horizon: int = 20,
                 success_reward: float = 5.0, wrong_attractor_cost: float = 2.0,
                 action_cost: float = 1.0, step_cost: float = 0.0, settle: int = 0):
        self.network = network
        self.attractors: Attractors = [[clean_state(s) for s in a] for a in (attractors or [])]
        self.perturbation = float(perturbation)
        self.prob_bits = int(prob_bits)
        self.horizon = int(horizon or 0)
        self.success_reward = float(success_reward)
        self.wrong_attractor_cost = float(wrong_attractor_cost)
        self.action_cost = float(action_cost)
        self.step_cost = float(step_cost)
        # step law: 0/1 = one synchronous update per env step; K >= 2 = the settle law (updates
        # until an attractor state, at most K; include/pbn_env.h "Step law")
        self.settle = int(settle or 0)
        if not 0 <= self.settle <= MAX_SETTLE:
            raise ValueError(f"settle must be in 0..{MAX_SETTLE}")
        if not 0 <= self.horizon <= 255:
            raise ValueError("horizon must be in 0..255 (0 = none)")
        if len(self.attractors) > MAX_ATTRACTORS:
            raise ValueError(f"at most {MAX_ATTRACTORS} attractors")
        n = network.n
        seen = {}
        for a, att in enumerate(self.attractors):
            if not att:
                raise ValueError(f"attractor {a} is empty")
            for s in att:
                if len(s) != n:
                    raise ValueError(f"attractor state of length {len(s)} for a {n}-node network")
                if s in seen and seen[s] != a:
                    raise ValueError(f"state {s} belongs to attractors {seen[s]} and {a}")
                seen[s] = a
        self._arrays = self._build()
        self._desc = self._make_desc()

    # -------------------------------------------------------------- helpers
    @property
    def n(self) -> int:
        return self.network.n

    @property
    def words(self) -> int:
        return self.network.words

    def reward_value(self, terminated: bool, wrong: bool, n_actions: int) -> float:
        return float(np.float32(self.success_reward * terminated - self.wrong_attractor_cost * wrong
                                - self.action_cost * n_actions - self.step_cost))

    def attractor_id(self, state: Sequence[int]) -> int:
        key = tuple(int(v) for v in state)
        for a, att in enumerate(self.attractors):
            if key in att:
                return a
        return -1

    def _build(self) -> dict:
        net = self.network
        arr = dict(net.descriptor_arrays(self.prob_bits))
        arr["perturb_cdf"] = perturbation_cdf(self.perturbation, net.n)
        starts, states = [0], []
        for att in self.attractors:
            for s in att:
                states.extend(net.pack(s))
            starts.append(starts[-1] + len(att))
        arr["attractor_start"] = np.asarray(starts, dtype=np.int32)
        arr["attractor_states"] = np.asarray(states if states else [0], dtype=np.uint32)
        n1 = net.n + 1
        tab = np.zeros(4 * n1, dtype=np.float32)
        for term in (0, 1):
            for wrong in (0, 1):
                for k in range(n1):
                    tab[(2 * term + wrong) * n1 + k] = self.reward_value(bool(term), bool(wrong), k)
        arr["reward_table"] = tab
        return {k: np.ascontiguousarray(v) for k, v in arr.items()}

    def _make_desc(self) -> PbnNetDesc:
        a = self._arrays
        d = PbnNetDesc()
        d.n_nodes = self.network.n
        d.n_funcs = int(a["func_arity"].shape[0])
        d.prob_bits = self.prob_bits
        d.horizon = self.horizon
        d.node_func_start = _ptr(a["node_func_start"])
        d.func_arity = _ptr(a["func_arity"])
        d.func_inputs = _ptr(a["func_inputs"])
        d.func_table = _ptr(a["func_table"])
        d.func_threshold = _ptr(a["func_threshold"])
        d.perturb_cdf = _ptr(a["perturb_cdf"])
        d.n_attractors = len(self.attractors)
        d.n_attractor_states = int(a["attractor_start"][-1])
        d.attractor_start = _ptr(a["attractor_start"])
        d.attractor_states = _ptr(a["attractor_states"])
        d.reward_table = _ptr(a["reward_table"])
        d.n_gates = int(a["n_gates"][0])
        d.gate_arity = _ptr(a["gate_arity"])
        d.gate_inputs = _ptr(a["gate_inputs"])
        d.gate_table = _ptr(a["gate_table"])
        d.settle_max = self.settle
        return d

    @property
    def desc(self) -> PbnNetDesc:
        return self._desc

    @property
    def arrays(self) -> dict:
        return self._arrays

    def describe(self) -> dict:
        return {
            "network": self.network.name, "n_nodes": self.n, "words": self.words,
            "n_attractors": len(self.attractors), "perturbation": self.perturbation,
            "prob_bits": self.prob_bits, "horizon": self.horizon, "settle": self.settle,
            "reward": {"success": self.success_reward, "wrong_attractor": self.wrong_attractor_cost,
                       "action": self.action_cost, "step": self.step_cost},
        }
