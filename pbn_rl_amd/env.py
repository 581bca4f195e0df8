"""PBNEnv: the gym-PBN environment surface, backed by the HIP step.

Drop-in for the env the reference builds with
``gym.make("gym-PBN/PBNEnv", N=, genes=, logic_functions=[, min_attractors=])``
(train_assa_BQN.py:121-124, model_tester.py:409-413) or
``gym.make("gym-PBN/BittnerMultiGeneral", N=28, horizon=20, min_attractors=7)``
(train_BDQ.py:50), exposing the attribute surface its callers use
(SURVEY.md Appendix A):

  reset() -> ((state, target), info)              bdq_model/__init__.py:161,204
  step(actions) -> (obs, reward, term, trunc, info)  bdq_model/__init__.py:177
      actions: list of ints / 0-d (CUDA) tensors, a tensor, an int, or []
      (0 = no-op, a > 0 flips node a-1, duplicates count once: bdq_model/__init__.py:76-84,176)
      the step law is the settle law by default (settle=DEFAULT_SETTLE = 64: intervene, then
      update synchronously until the state is an attractor state, at most 64 updates;
      include/pbn_env.h "Step law"), the law the reference's recorded evaluation
      data/results/pbn_33_3.pkl pins (model_tester.py:616-626; tests/test_bn_pin.py);
      settle=0 selects one synchronous update per step (the unit bench.py's headline counts)
  observation_space.shape[0]                      train_BDQ.py:82
  attracting_states, all_attractors, real_attractors      bdq_model/__init__.py:60,182
  state_attractor_id, target_attractor_id         bdq_model/__init__.py:180
  rework_probas(ep_len=None)                      bdq_model/__init__.py:203
  is_attracting_state(s), in_target(s), setTarget(a), render()   model_tester.py:611-625,
                                                  graph_classifier/__init__.py:129
  graph.setState(s), graph.nodes[i].index / .predictors, graph.getNodeByID(id)
                                                  gbdq_model/__init__.py:264-274
  env.env.env chain, close()                      train_pbn_BQN.py:90, train_BDQ.py:116

One PBNEnv is one env (gym semantics: no autoreset; callers call reset()).  It
runs on the GPU as env 0 of a VectorPBNEnv group.  Between steps the env lives
in pinned host memory mapped into the device (pbn_host_buffer, _HostGroup): a
step is one pbn_step launch with n_envs = 1 on those pointers and one stream
synchronisation, no copies and no torch tensors.  Use VectorPBNEnv for batched
rollouts.
"""
from __future__ import annotations

import warnings
from typing import List, Optional, Sequence, Tuple, Union

import numpy as np
import torch

from . import _lib
from .attractors import Attractors, clean_state, find_attractors, load_attractors
from .network import Network, load_network
from .spec import NO_TARGET, EnvSpec
from .vector_env import VectorPBNEnv

__all__ = ["PBNEnv", "ControlPBNEnv", "make", "Box", "MultiDiscrete", "DEFAULT_SETTLE"]

# The facade's step law: the settle law with a cap of 64 synchronous updates per env step.  The
# reference's recorded bb33 evaluation (data/results/pbn_33_3.pkl, model_tester.py:587-658)
# needs at least two updates after an intervention and is reproduced for every cap >= 2; the
# one-update law (settle=0) fails it under every attractor order (tests/test_bn_pin.py).
DEFAULT_SETTLE = 64


class Box:
    def __init__(self, low, high, shape, dtype=np.int8):
        self.low, self.high, self.shape, self.dtype = low, high, tuple(shape), dtype

    def sample(self, rng=None):
        rng = rng or np.random.default_rng()
        return rng.integers(self.low, self.high + 1, size=self.shape).astype(self.dtype)


class MultiDiscrete:
    def __init__(self, nvec):
        self.nvec = np.asarray(nvec)
        self.shape = self.nvec.shape

    def sample(self, rng=None):
        rng = rng or np.random.default_rng()
        return rng.integers(0, self.nvec)


class _Node:
    """gym-PBN style node: ``index``, ``ID`` and ``predictors = [(IDs, A, COD)]``."""

    def __init__(self, index: int, name: str, predictors):
        self.index = index
        self.ID = name
        self.name = name
        self.predictors = predictors


class _Graph:
    def __init__(self, env: "PBNEnv"):
        self._env = env
        net = env.spec.network
        thr = net.thresholds(env.spec.prob_bits)
        self.nodes: List[_Node] = []
        for i, fl in enumerate(net.nodes):
            preds, prev = [], 0
            for f, c in zip(fl, thr[i]):
                A = np.array([(f.table >> m) & 1 for m in range(1 << f.arity)], dtype=np.int8)
                preds.append((tuple(net.genes[g] for g in f.inputs), A, (c - prev) / float(1 << env.spec.prob_bits)))
                prev = c
            self.nodes.append(_Node(i, net.genes[i], preds))
        self._by_id = {n.ID: n for n in self.nodes}

    def getNodeByID(self, ident):
        return self._by_id[ident]

    def setState(self, state: Sequence) -> None:
        self._env._set_state(clean_state(state))

    def getState(self):
        return self._env.render()

    def genSTG(self, **reached):
        """State-transition graph {state: set(successor states)} (print_graph.py:15-34): every
        state for networks of at most 20 nodes; beyond that the region GPU chains reach from
        random starts, closed under successors, with its exact successor relation
        (``discovery.reached_stg``; keyword arguments go to it)."""
        from .attractors import _successor_options  # exhaustive, N <= 20
        net = self._env.spec.network
        if net.n > 20:
            from .discovery import reached_stg
            return reached_stg(net, prob_bits=self._env.spec.prob_bits, device=self._env._venv.device, **reached)
        stg = {}
        for s in range(1 << net.n):
            opts = _successor_options(net, s, self._env.spec.prob_bits)
            nexts = [0]
            for i, vals in enumerate(opts):
                nexts = [x | (v << i) for x in nexts for v in vals]
            stg[tuple(net.unpack([s]))] = {tuple(net.unpack([x])) for x in nexts}
        return stg


class _HostGroup:
    """The facade's env in pinned, device-mapped host memory (pbn_host_buffer, ABI 9): two state
    buffers (ping-pong), the flip mask, reward, flags, target and step count, each as a numpy view
    (host side) and a device address (the kernel's side).  pbn_reset / pbn_step run on it with
    n_envs = n (1: the other 31 envs of the group are not computed into the step's cost, in
    particular not into the settle law's wave-wide loop)."""

    _LAYOUT = (("state0", 4, 1), ("state1", 4, 1), ("flip", 4, 1), ("reward", 4, 0), ("flags", 1, 0),
               ("target", 1, 0), ("t", 1, 0))

    def __init__(self, words: int, n: int = 1):
        import ctypes
        L = _lib.load()
        self.words, self.n = words, n
        offs, off = {}, 0
        for name, size, per_word in self._LAYOUT:
            offs[name] = off
            off += ((size * n * (words if per_word else 1)) + 15) & ~15
        h, d = ctypes.c_void_p(), ctypes.c_void_p()
        _lib.check(L.pbn_host_buffer(off, ctypes.byref(h), ctypes.byref(d)), "pbn_host_buffer")
        self._h, self._d, self.bytes = h.value, d.value, off
        raw = np.ctypeslib.as_array((ctypes.c_uint8 * off).from_address(self._h))
        dt = {"reward": np.float32, "flags": np.uint8, "target": np.uint8, "t": np.uint8}
        self.view, self.dev = {}, {}
        for name, size, per_word in self._LAYOUT:
            o = offs[name]
            nb = size * n * (words if per_word else 1)
            v = raw[o:o + nb].view(dt.get(name, np.uint32))
            self.view[name] = v.reshape(words, n) if per_word else v
            self.dev[name] = self._d + o
        self.cur = 0   # state{cur} holds the current state

    def state(self) -> np.ndarray:
        return self.view[f"state{self.cur}"]

    def free(self) -> None:
        if getattr(self, "_h", None):
            _lib.load().pbn_host_buffer_free(self._h)
            self._h = None


class PBNEnv:
    metadata = {"render_modes": ["human", "PBN"]}

    def __init__(self, N: Optional[int] = None, genes: Optional[Sequence[str]] = None, logic_functions=None,
                 min_attractors: Optional[int] = None, *, network: Union[str, Network, None] = None,
                 attractors: Optional[Attractors] = None, horizon: int = 20, perturbation: float = 0.01,
                 prob_bits: int = 16, seed: Optional[int] = None, device=None, render_mode=None,
                 success_reward: float = 5.0, wrong_attractor_cost: float = 2.0, action_cost: float = 1.0,
                 step_cost: float = 0.0, name: Optional[str] = None, grow_attractors: bool = True,
                 discovery: Optional[dict] = None, settle: int = DEFAULT_SETTLE):
        if isinstance(network, str):
            if attractors is None:
                attractors = load_attractors(network)
            network = load_network(network)
        elif network is None:
            if genes is None or logic_functions is None:
                raise ValueError("give network= or genes= and logic_functions=")
            network = Network.from_logic_functions(genes, logic_functions, name=name or "pbn")
        if N is not None and N != network.n:
            raise ValueError(f"N={N} but the network has {network.n} nodes")
        if attractors is None:
            # exhaustive STG search while it is cheap; beyond that, GPU simulation + exact
            # verification (discovery.py); both return bottom SCCs (print_graph.py:15-34)
            if network.n <= 16:
                attractors = find_attractors(network, prob_bits=prob_bits)
            else:
                from .discovery import discover_attractors_escalating
                attractors = discover_attractors_escalating(network, prob_bits=prob_bits, device=device,
                                                            **(discovery or {}))
        if not attractors:
            raise ValueError(f"{network.name}: no attractor found (no targets or terminal states); pass "
                             f"attractors= or discovery= (chains/burn_in) explicitly")
        if min_attractors is not None and len(attractors) < min_attractors:
            warnings.warn(f"network has {len(attractors)} attractors < min_attractors={min_attractors}")
        self._spec_kwargs = dict(perturbation=perturbation, prob_bits=prob_bits, horizon=horizon,
                                 success_reward=success_reward, wrong_attractor_cost=wrong_attractor_cost,
                                 action_cost=action_cost, step_cost=step_cost, settle=settle)
        self.spec = EnvSpec(network, attractors, **self._spec_kwargs)
        self.N = network.n
        self.render_mode = render_mode
        self._seed = int(seed if seed is not None else np.random.SeedSequence().entropy % (1 << 63))
        self._venv = VectorPBNEnv(self.spec, 1, seed=self._seed, device=device, autoreset=False)
        self.observation_space = Box(0, 1, (self.N,))
        self.action_space = MultiDiscrete([self.N + 1] * 3)
        self.discrete_action_space = self.action_space
        self.graph = _Graph(self)
        self.all_attractors: List[List[Tuple[int, ...]]] = [list(a) for a in self.spec.attractors]
        # the attractor set the env was built with; all_attractors may grow (grow())
        self.real_attractors = [list(a) for a in self.spec.attractors]
        self.attracting_states = [s for a in self.all_attractors for s in a]
        self.state_attractor_id = -1
        self.target_attractor_id = -1
        self.target = None
        self.n_steps = 0
        self.target_nodes: List[int] = []
        self.control_nodes = list(range(self.N))
        self._ep_lens: List[int] = []
        # attractor growth (bdq_model/__init__.py:182-184): states revisited outside the known
        # attractors are verified as bottom SCCs (discovery.bottom_sccs) at episode ends
        self.grow_attractors = grow_attractors
        self.visit_cap = 1 << 16     # bound on the host-side visit table (packed-state keys)
        self._visits: dict = {}
        self._checked: set = set()
        # rework_probas (bdq_model/__init__.py:203): per (start, target) pair weights
        self._pair_len: Optional[np.ndarray] = None
        self._rng = np.random.default_rng(self._seed)
        # the group in device-mapped host memory between steps (_HostGroup); ``_hg_live``: it, not
        # the VectorPBNEnv's device tensors, holds the current state / target / step count
        self._hg: Optional[_HostGroup] = None
        self._hg_live = False
        self._bit = np.arange(self.N)
        self._bit_word, self._bit_pos = self._bit >> 5, (self._bit & 31).astype(np.uint32)

    # gymnasium wrapper chain compatibility (env.env.env, env.unwrapped)
    @property
    def env(self):
        return self

    @property
    def unwrapped(self):
        return self

    # ---------------------------------------------------------------- core
    def _unpack(self, words: np.ndarray) -> np.ndarray:
        """bits of env 0's state words (node i = bit i & 31 of word i >> 5, Network.pack)"""
        return ((words[self._bit_word] >> self._bit_pos) & 1).astype(np.int64)

    def _read_state(self) -> np.ndarray:
        if self._hg_live:
            return self._unpack(self._hg.state()[:, 0])
        w = self._venv.state[:, 0].cpu().numpy().view(np.uint32)
        return np.array(self.spec.network.unpack(list(w)), dtype=np.int64)

    def _to_device(self) -> None:
        """The host group's state / target / step count back into the VectorPBNEnv (before any
        operation on its tensors)."""
        if not self._hg_live:
            return
        hg, venv = self._hg, self._venv
        n = hg.n
        venv.state[:, :n].copy_(torch.from_numpy(hg.state().view(np.int32).copy()))
        venv.target[:n].copy_(torch.from_numpy(hg.view["target"].copy()))
        venv.t[:n].copy_(torch.from_numpy(hg.view["t"].copy()))
        self._hg_live = False

    def _to_host(self) -> None:
        """The VectorPBNEnv's group into the host group (first step after reset / setState)."""
        if self._hg is None:   # env 0 alone: pbn_reset / pbn_step take n_envs = 1 (ABI 9)
            self._hg = _HostGroup(self.spec.words, 1)
        hg, venv = self._hg, self._venv
        n = hg.n
        hg.state()[:] = venv.state[:, :n].cpu().numpy().view(np.uint32)
        hg.view["target"][:] = venv.target[:n].cpu().numpy()
        hg.view["t"][:] = venv.t[:n].cpu().numpy()
        hg.view["flip"][:] = 0
        self._hg_live = True

    def _set_state(self, bits: Tuple[int, ...]) -> None:
        words = np.array(self.spec.network.pack(bits), dtype=np.uint32)
        if self._hg_live:
            self._hg.state()[:, 0] = words
            return
        self._venv.state[:, :1].copy_(torch.tensor(words.view(np.int32)[:, None], device=self._venv.device))

    def _set_target_id(self, idx: int) -> None:
        if self._hg_live:
            self._hg.view["target"][0] = idx
        else:
            self._venv.target[:1].fill_(idx)

    def reset(self, seed: Optional[int] = None, options=None):
        if seed is not None:
            self._seed = int(seed)
        venv = self._venv
        if self._hg is not None:   # pbn_reset straight into the host group (as VectorPBNEnv.reset)
            hg = self._hg
            venv.seed = self._seed & 0xFFFFFFFFFFFFFFFF
            L = _lib.load()
            stream = venv._stream()
            _lib.check(L.pbn_reset(venv.net.handle, venv.seed, venv.step_index, venv.env_offset, hg.n,
                                   hg.dev[f"state{hg.cur}"], hg.dev["target"], hg.dev["t"], stream), "pbn_reset")
            _lib.check(L.pbn_stream_sync(stream), "pbn_stream_sync")
            venv.step_index += 1
            self._hg_live = True
        else:
            self._hg_live = False
            venv.reset(seed=self._seed)
        if self._pair_len is not None and len(self.all_attractors) >= 2:
            self._reset_reweighted()
        state = self._read_state()
        tgt = int(self._hg.view["target"][0]) if self._hg_live else int(venv.target[0].item())
        self.target_attractor_id = tgt if tgt != NO_TARGET else -1
        self.state_attractor_id = self.spec.attractor_id(state)
        self.target = list(self.all_attractors[tgt][0]) if tgt != NO_TARGET else None
        target_vec = np.array(self.target if self.target is not None else [0] * self.N, dtype=np.int64)
        self.n_steps = 0
        return (state, target_vec), {"target_attractor": self.target_attractor_id,
                                     "state_attractor": self.state_attractor_id}

    @staticmethod
    def _actions(action) -> List[int]:
        if action is None:
            return []
        if isinstance(action, torch.Tensor):
            return [int(x) for x in action.reshape(-1).tolist()]
        if isinstance(action, np.ndarray):
            return [int(x) for x in action.reshape(-1)]
        if isinstance(action, (int, np.integer)):
            return [int(action)]
        return [int(x.item()) if isinstance(x, torch.Tensor) else int(x) for x in action]

    def step(self, action):
        acts = self._actions(action)
        bits = [0] * self.N
        for a in acts:
            if not 0 <= a <= self.N:
                raise ValueError(f"action {a} outside [0, {self.N}]")
            if a > 0:
                bits[a - 1] = 1
        venv = self._venv
        if not self._hg_live:
            self._to_host()
        hg = self._hg
        hg.view["flip"][:, 0] = np.array(self.spec.network.pack(bits), dtype=np.uint32)
        # one launch on the mapped group, one synchronisation, no copies (pbn_step's arguments as
        # VectorPBNEnv.step_flipmask passes them: same seed, step index and env range)
        L = _lib.load()
        nxt = 1 - hg.cur
        stream = venv._stream()
        _lib.check(L.pbn_step(venv.net.handle, venv.seed, venv.step_index, venv.env_offset, hg.n,
                              _lib.MODE_AUTORESET if venv.autoreset else 0, hg.dev[f"state{hg.cur}"], hg.dev["flip"],
                              hg.dev["target"], hg.dev["t"], hg.dev[f"state{nxt}"], None, hg.dev["reward"],
                              hg.dev["flags"], stream), "pbn_step")
        _lib.check(L.pbn_stream_sync(stream), "pbn_stream_sync")
        venv.step_index += 1
        hg.cur = nxt
        words = hg.state()[:, 0]
        fl = int(hg.view["flags"][0])
        r = float(hg.view["reward"][0])
        obs = self._unpack(words)
        self.n_steps += 1
        if self.grow_attractors and not fl & _lib.FLAG_IN_ATTRACTOR:
            key = int.from_bytes(words.tobytes(), "little")
            self._visits[key] = self._visits.get(key, 0) + 1
            if len(self._visits) > self.visit_cap:
                self._prune_visits()
        info = {"perturbed": bool(fl & _lib.FLAG_PERTURBED), "in_attractor": bool(fl & _lib.FLAG_IN_ATTRACTOR),
                "unsettled": bool(fl & _lib.FLAG_UNSETTLED), "flags": fl}
        return obs, r, bool(fl & _lib.FLAG_TERMINATED), bool(fl & _lib.FLAG_TRUNCATED), info

    # ------------------------------------------------------ attribute surface
    def render(self):
        return list(self._read_state())

    def is_attracting_state(self, state) -> bool:
        return self.spec.attractor_id(clean_state(state)) >= 0

    def in_target(self, state) -> bool:
        if self.target_attractor_id < 0:
            return False
        return tuple(clean_state(state)) in set(self.all_attractors[self.target_attractor_id])

    def setTarget(self, target) -> None:
        """target: an attractor (list of states), one state, or an attractor index."""
        if isinstance(target, (int, np.integer)):
            idx = int(target)
        else:
            first = target[0] if len(target) and isinstance(target[0], (list, tuple, np.ndarray)) else target
            idx = self.spec.attractor_id(clean_state(first))
            if idx < 0:
                raise ValueError("target is not a state of a known attractor")
        self.target_attractor_id = idx
        self.target = list(self.all_attractors[idx][0])
        self._set_target_id(idx)

    def rework_probas(self, ep_len: Optional[int] = None) -> None:
        """Called by the learner after every episode (bdq_model/__init__.py:203;
        graph_classifier/__init__.py:155 without an argument).  The fork's rule is unavailable
        (SURVEY.md 0.2); this build's documented rule, a curriculum over (start, target) pairs:

        * ``ep_len`` updates the finished episode's pair: its weight is the running mean of its
          episode lengths (every pair starts at the horizon), so pairs that take long or time
          out are drawn more often;
        * from the first call on, ``reset()`` draws the pair with probability proportional to
          its weight (target != start), from a host generator seeded with the env seed, and
          places the start attractor's first state; before it, reset draws are the device's
          uniform ones (keyed by seed, env and step).

        It also runs the attractor-growth check (``grow()``) at the episode end."""
        A = len(self.all_attractors)
        if ep_len is not None:
            self._ep_lens.append(int(ep_len))
            if A >= 2:
                if self._pair_len is None or self._pair_len.shape[0] != A:
                    old = self._pair_len
                    self._pair_len = np.full((A, A, 2), [float(self.spec.horizon or 20), 1.0])
                    if old is not None:
                        k = old.shape[0]
                        self._pair_len[:k, :k] = old
                s, t = self.state_attractor_id, self.target_attractor_id
                if 0 <= s < A and 0 <= t < A:
                    tot, cnt = self._pair_len[s, t]
                    self._pair_len[s, t] = (tot + float(ep_len), cnt + 1)
        if self.grow_attractors:
            self.grow()

    def pair_weights(self) -> Optional[np.ndarray]:
        """(A, A) reset probabilities of the rework_probas curriculum (None before its first call)."""
        if self._pair_len is None:
            return None
        w = self._pair_len[:, :, 0] / self._pair_len[:, :, 1]
        np.fill_diagonal(w, 0.0)
        return w / w.sum()

    def _reset_reweighted(self) -> None:
        w = self.pair_weights().reshape(-1)
        k = int(self._rng.choice(w.size, p=w))
        A = len(self.all_attractors)
        s, t = divmod(k, A)
        self._set_state(self.all_attractors[s][0])
        self._set_target_id(t)

    def grow(self, min_visits: int = 2, max_states: int = 1 << 14) -> int:
        """Attractor growth (bdq_model/__init__.py:182-184 re-raises epsilon when
        ``len(env.all_attractors)`` grows): states the env revisited outside every known attractor
        are closed under the successor relation and verified as bottom SCCs of the STG
        (``discovery.bottom_sccs``, the print_graph.py:15-34 definition); new ones are appended
        to ``all_attractors``/``attracting_states`` and become reward/target states on the
        device.  Returns the number added."""
        from .discovery import bottom_sccs
        from .spec import MAX_ATTRACTORS

        cand = [k for k, c in self._visits.items() if c >= min_visits and k not in self._checked]
        if not cand or len(self.all_attractors) >= MAX_ATTRACTORS:
            return 0
        if len(self._checked) + len(cand) > self.visit_cap:
            self._checked.clear()
        self._checked.update(cand)
        W = self.spec.words
        rows = np.array([self.spec.network.unpack([(k >> (32 * w)) & 0xFFFFFFFF for w in range(W)]) for k in cand],
                        dtype=np.uint8)
        found = bottom_sccs(self.spec.network, rows, prob_bits=self.spec.prob_bits, max_states=max_states)
        known = {s for a in self.all_attractors for s in a}
        new = [a for a in found if not any(s in known for s in a)]
        new = new[:MAX_ATTRACTORS - len(self.all_attractors)]
        for k in cand:   # checked: their visit counts are no longer needed
            self._visits.pop(k, None)
        if not new:
            return 0
        self.all_attractors.extend([list(a) for a in new])
        self.attracting_states = [s for a in self.all_attractors for s in a]
        self.spec = EnvSpec(self.spec.network, self.all_attractors, **self._spec_kwargs)
        self._to_device()
        self._venv.set_spec(self.spec)
        return len(new)

    def _prune_visits(self) -> None:
        """Keep the visit table within visit_cap: drop the states seen once (a revisit is what
        makes a candidate), then, if still full, the oldest half."""
        self._visits = {k: c for k, c in self._visits.items() if c > 1}
        if len(self._visits) > self.visit_cap // 2:
            keys = list(self._visits)
            for k in keys[:len(keys) // 2]:
                del self._visits[k]

    def close(self) -> None:
        self._to_device()
        if self._hg is not None:
            self._hg.free()
            self._hg = None
        self._venv.close()


class ControlPBNEnv(PBNEnv):
    """gym-PBN/ControlPBNEnv (train_control_gbdq.py:45-72): PBNEnv whose action is one binary
    value per control node (control_gbdq_model/__init__.py:35,169: action_count =
    len(env.control_nodes), 2 choices per branch).  Control node c_k is set to action[k] in s1
    before the synchronous update: the flip mask is (s XOR v) on the control nodes, so the step
    kernel runs unchanged and the action cost counts the control nodes that changed.  This is
    an assumed semantics (PBNControlMultiEnv is absent; unpinned).

    Control node indices outside [0, N) are kept in ``control_nodes`` (the agent sizes its
    action from its length) but their action entries are ignored, with a warning: the reference
    script lists node 14 of a 14-gene network."""

    def __init__(self, N: Optional[int] = None, genes: Optional[Sequence[str]] = None, logic_functions=None,
                 min_attractors: Optional[int] = None, *, control_nodes: Sequence[int] = (), **kwargs):
        super().__init__(N, genes, logic_functions, min_attractors, **kwargs)
        self.control_nodes = [int(c) for c in control_nodes]
        bad = [c for c in self.control_nodes if not 0 <= c < self.N]
        if bad:
            warnings.warn(f"control nodes {bad} are outside [0, {self.N}) and will be ignored")
        self._ctrl = [(k, c) for k, c in enumerate(self.control_nodes) if 0 <= c < self.N]
        self.action_space = MultiDiscrete([2] * len(self.control_nodes))
        self.discrete_action_space = self.action_space

    def step(self, action):
        vals = self._actions(action)
        if len(vals) != len(self.control_nodes):
            raise ValueError(f"expected {len(self.control_nodes)} control values, got {len(vals)}")
        state = self._read_state()
        flips = [c + 1 for k, c in self._ctrl if (int(vals[k]) & 1) != int(state[c])]
        return super().step(flips)


def make(env_id: str, **kwargs):
    """Minimal stand-in for gymnasium.make over the env ids the reference uses."""
    key = env_id.split("/")[-1]
    if key == "PBNEnv":
        return PBNEnv(**kwargs)
    if key == "ControlPBNEnv":
        return ControlPBNEnv(**kwargs)
    if key.startswith("BittnerMultiGeneral") or key.startswith("BittnerMulti-") or key.startswith("Bittner-"):
        n = kwargs.pop("N", None)
        if n is None:
            digits = "".join(c for c in key.split("-")[-1] if c.isdigit())
            n = int(digits) if digits else 28
        bundled = {7: "pbn7", 10: "pbn10", 28: "pbn28", 70: "pbn70"}
        if n not in bundled:
            raise ValueError(f"no bundled Bittner network with {n} nodes (have {sorted(bundled)})")
        return PBNEnv(network=bundled[n], **kwargs)
    raise ValueError(f"unknown env id {env_id!r}")
