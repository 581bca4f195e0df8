"""VectorPBNEnv: a batch of PBN envs resident in HBM, stepped by libpbn_env.so.

This is the batched form of the gym-PBN env the reference steps one frame at
a time (bdq_model/__init__.py:172-177).  All buffers are torch tensors on one
GPU in the SoA layout of include/pbn_env.h (uint32 words stored as int32);
every step is one ``pbn_step`` launch on the current torch stream, with no
host synchronisation.  Buffers are padded to a multiple of 32 envs (the
kernel's group size); the padding envs are real envs nobody reads.
"""
from __future__ import annotations

import ctypes
from typing import Optional, Sequence, Tuple, Union

import torch

from . import _lib
from .spec import EnvSpec

__all__ = ["VectorPBNEnv", "actions_to_flipmask", "control_to_flipmask", "unpack_states", "pack_states"]


def _round32(n: int) -> int:
    return (n + 31) // 32 * 32


def actions_to_flipmask(actions: torch.Tensor, n_nodes: int, check: bool = True) -> torch.Tensor:
    """(n, k) ints in [0, N] -> (W, n) int32 flip masks; 0 = no-op, a > 0 flips node a-1
    once however often it is repeated (bdq_model/__init__.py:81-84,176).  ``check=False``
    skips the range check (a host sync; out-of-range actions then flip nothing), for
    graph-captured loops."""
    if actions.dim() == 1:
        actions = actions[:, None]
    n = actions.shape[0]
    W = (n_nodes + 31) // 32
    a = actions.to(torch.int64)
    if check and bool(((a < 0) | (a > n_nodes)).any()):
        raise ValueError(f"actions must be in [0, {n_nodes}]")
    node = torch.arange(1, n_nodes + 1, device=a.device)
    hit = (a[:, :, None] == node[None, None, :]).any(dim=1)          # (n, N)
    pad = torch.zeros(n, 32 * W, dtype=torch.int64, device=a.device)
    pad[:, :n_nodes] = hit.to(torch.int64)
    weights = (torch.ones(32, dtype=torch.int64, device=a.device) << torch.arange(32, device=a.device))
    words = (pad.view(n, W, 32) * weights).sum(dim=2)                  # (n, W) in [0, 2^32)
    words = torch.where(words >= 2 ** 31, words - 2 ** 32, words)
    return words.to(torch.int32).t().contiguous()


def control_to_flipmask(state: torch.Tensor, values: torch.Tensor, control_nodes: Sequence[int],
                        n_nodes: int) -> torch.Tensor:
    """The ControlPBNEnv action form (train_control_gbdq.py:45-72, control_gbdq_model/__init__.py:
    35,169): one binary action per control node.  Assumed semantics (gym_PBN's
    PBNControlMultiEnv is absent, so this is unpinned): control node c_k takes the value
    values[:, k] in s1, i.e. the flip mask is (s XOR v) restricted to the control nodes, and the
    step then runs unchanged.  state (W, n) int32 words, values (n, C) 0/1 -> (W, n) int32."""
    W, n = state.shape
    if W != (n_nodes + 31) // 32:
        raise ValueError(f"state has {W} words, {n_nodes} nodes need {(n_nodes + 31) // 32}")
    if values.dim() == 1:
        values = values[None, :]
    if values.shape != (n, len(control_nodes)):
        raise ValueError(f"values must have shape {(n, len(control_nodes))}")
    v = values.to(device=state.device, dtype=torch.int64) & 1
    vw = torch.zeros(W, n, dtype=torch.int64, device=state.device)
    cw = [0] * W
    for k, c in enumerate(control_nodes):
        if not 0 <= c < n_nodes:
            raise ValueError(f"control node {c} outside [0, {n_nodes})")
        vw[c >> 5] |= v[:, k] << (c & 31)
        cw[c >> 5] |= 1 << (c & 31)
    vw = torch.where(vw >= 2 ** 31, vw - 2 ** 32, vw).to(torch.int32)
    cm = torch.tensor([m - (1 << 32) if m >= 1 << 31 else m for m in cw], dtype=torch.int32,
                      device=state.device)[:, None]
    return (state ^ vw) & cm


def unpack_states(words: torch.Tensor, n_nodes: int) -> torch.Tensor:
    """(W, n) int32 words -> (n, N) uint8 bits (node i = bit i)."""
    W, n = words.shape
    shifts = torch.arange(32, device=words.device, dtype=torch.int32)
    bits = (words.t()[:, :, None] >> shifts[None, None, :]) & 1     # (n, W, 32)
    return bits.reshape(n, 32 * W)[:, :n_nodes].to(torch.uint8)


def pack_states(bits: torch.Tensor, n_nodes: int) -> torch.Tensor:
    """(n, N) 0/1 -> (W, n) int32 words."""
    n = bits.shape[0]
    W = (n_nodes + 31) // 32
    pad = torch.zeros(n, 32 * W, dtype=torch.int64, device=bits.device)
    pad[:, :n_nodes] = bits.to(torch.int64) & 1
    weights = torch.ones(32, dtype=torch.int64, device=bits.device) << torch.arange(32, device=bits.device)
    words = (pad.view(n, W, 32) * weights).sum(dim=2)
    words = torch.where(words >= 2 ** 31, words - 2 ** 32, words)
    return words.to(torch.int32).t().contiguous()


class VectorPBNEnv:
    """``num_envs`` PBN envs on ``device``; env ids ``env_offset .. env_offset+num_envs``.

    step() consumes either a (W, n) flip-mask tensor, an (n, k) action tensor,
    or nothing (``random_actions=True``: 3 uniform actions per env drawn in-kernel,
    the synthetic explore policy of bdq_model/__init__.py:76).
    """

    def __init__(self, spec: EnvSpec, num_envs: int, *, seed: int = 0, device: Union[str, torch.device, None] = None,
                 env_offset: int = 0, autoreset: bool = True, keep_final_state: bool = True):
        if not torch.cuda.is_available():
            raise _lib.PbnError("VectorPBNEnv needs a ROCm GPU (libpbn_env.so has no CPU path)")
        if env_offset % 32:
            raise ValueError("env_offset must be a multiple of 32")
        self.spec = spec
        self.device = torch.device(device if device is not None else f"cuda:{torch.cuda.current_device()}")
        self.num_envs = int(num_envs)
        self.n_alloc = _round32(self.num_envs)
        self.env_offset = int(env_offset)
        self.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
        self.autoreset = autoreset
        self.keep_final_state = keep_final_state
        self.n_nodes = spec.n
        self.words = spec.words
        with torch.cuda.device(self.device):
            self.net = _lib.NetHandle(spec)
        W, n = self.words, self.n_alloc
        dev = self.device
        z32 = lambda *s: torch.zeros(*s, dtype=torch.int32, device=dev)  # noqa: E731
        self.state = z32(W, n)
        self._state_next = z32(W, n)
        self.flipmask = z32(W, n)
        self.final_state = z32(W, n) if keep_final_state else None
        self.target = torch.zeros(n, dtype=torch.uint8, device=dev)
        self.t = torch.zeros(n, dtype=torch.uint8, device=dev)
        self.reward = torch.zeros(n, dtype=torch.float32, device=dev)
        self.flags = torch.zeros(n, dtype=torch.uint8, device=dev)
        self.step_index = 0      # global step counter: the RNG's time coordinate

    # ------------------------------------------------------------ internals
    def _stream(self) -> int:
        return torch.cuda.current_stream(self.device).cuda_stream

    def reset(self, seed: Optional[int] = None) -> Tuple[torch.Tensor, torch.Tensor]:
        if seed is not None:
            self.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
        L = _lib.load()
        with torch.cuda.device(self.device):
            _lib.check(L.pbn_reset(self.net.handle, self.seed, self.step_index, self.env_offset, self.n_alloc,
                                   self.state.data_ptr(), self.target.data_ptr(), self.t.data_ptr(),
                                   self._stream()), "pbn_reset")
        self.step_index += 1
        return self.state[:, : self.num_envs], self.target[: self.num_envs]

    def step_flipmask(self, flipmask: Optional[torch.Tensor] = None, random_actions: bool = False,
                      use_current: bool = False):
        """One transition for every env; returns views (state', reward, flags).
        ``use_current``: step with what ``self.flipmask`` already holds (e.g. written by
        pbn_q_to_flipmask), for all ``n_alloc`` envs."""
        L = _lib.load()
        mode = _lib.MODE_AUTORESET if self.autoreset else 0
        if random_actions:
            mode |= _lib.MODE_RANDOM_ACTIONS
        elif use_current:
            pass
        elif flipmask is not None:
            if flipmask.shape != (self.words, self.num_envs):
                raise ValueError(f"flipmask must have shape {(self.words, self.num_envs)}")
            self.flipmask[:, : self.num_envs].copy_(flipmask)
            if self.n_alloc > self.num_envs:
                self.flipmask[:, self.num_envs:].zero_()
        else:
            self.flipmask.zero_()
        fs = self.final_state.data_ptr() if self.final_state is not None else None
        with torch.cuda.device(self.device):
            _lib.check(L.pbn_step(self.net.handle, self.seed, self.step_index, self.env_offset, self.n_alloc, mode,
                                  self.state.data_ptr(), self.flipmask.data_ptr(), self.target.data_ptr(),
                                  self.t.data_ptr(), self._state_next.data_ptr(), fs, self.reward.data_ptr(),
                                  self.flags.data_ptr(), self._stream()), "pbn_step")
        self.step_index += 1
        self.state, self._state_next = self._state_next, self.state
        k = self.num_envs
        return self.state[:, :k], self.reward[:k], self.flags[:k]

    def step_control(self, values: torch.Tensor, control_nodes: Sequence[int]):
        """One transition with the ControlPBNEnv action form: control node c_k set to
        values[:, k] (0/1, shape (num_envs, C)) before the update (see control_to_flipmask)."""
        fm = control_to_flipmask(self.state[:, : self.num_envs], values, control_nodes, self.n_nodes)
        return self.step_flipmask(fm)

    def step_flipmask_dev(self, step_t: torch.Tensor, copy_back: bool = True):
        """``step_flipmask(use_current=True)`` through ``pbn_step_dev``: the step index is read
        from the int64 device tensor ``step_t`` when the kernel runs, and the new state is
        copied back into ``self.state`` (no buffer swap), so the call can be captured in a
        hipGraph and replayed.  Neither ``step_t`` nor ``step_index`` is advanced here: the
        caller advances ``step_t`` on the stream and mirrors it in ``step_index``.  ``copy_back=False``
        leaves the new state in ``_state_next`` for the caller to move (BDQLearner's captured frame
        does it inside its ring store) and returns it instead of ``state``."""
        if step_t.dtype != torch.int64 or step_t.device != self.device or step_t.numel() != 1:
            raise ValueError("step_t must be a one-element int64 tensor on the env's device")
        L = _lib.load()
        mode = _lib.MODE_AUTORESET if self.autoreset else 0
        fs = self.final_state.data_ptr() if self.final_state is not None else None
        with torch.cuda.device(self.device):
            _lib.check(L.pbn_step_dev(self.net.handle, self.seed, step_t.data_ptr(), self.env_offset, self.n_alloc,
                                      mode, self.state.data_ptr(), self.flipmask.data_ptr(), self.target.data_ptr(),
                                      self.t.data_ptr(), self._state_next.data_ptr(), fs, self.reward.data_ptr(),
                                      self.flags.data_ptr(), self._stream()), "pbn_step_dev")
        k = self.num_envs
        if not copy_back:
            return self._state_next[:, :k], self.reward[:k], self.flags[:k]
        self.state.copy_(self._state_next)
        return self.state[:, :k], self.reward[:k], self.flags[:k]

    def step_flipmask_dev_store(self, step_t: torch.Tensor, ring) -> None:
        """``step_flipmask_dev`` that also writes the step's transitions into a replay ring
        (``pbn_step_dev_store``, one launch where the step and ``pbn_replay_store`` were two; the
        one-update law only).  ``ring``: an ``_lib.RingStore``.  The state is stepped in place."""
        if step_t.dtype != torch.int64 or step_t.device != self.device or step_t.numel() != 1:
            raise ValueError("step_t must be a one-element int64 tensor on the env's device")
        L = _lib.load()
        mode = _lib.MODE_AUTORESET if self.autoreset else 0
        fs = self.final_state.data_ptr() if self.final_state is not None else None
        with torch.cuda.device(self.device):
            _lib.check(L.pbn_step_dev_store(self.net.handle, self.seed, step_t.data_ptr(), self.env_offset,
                                            self.n_alloc, mode, self.state.data_ptr(), self.flipmask.data_ptr(),
                                            self.target.data_ptr(), self.t.data_ptr(), fs, self.reward.data_ptr(),
                                            self.flags.data_ptr(), ctypes.byref(ring), self._stream()),
                       "pbn_step_dev_store")

    def rollout_buffers(self, n_steps: int, keep_obs: bool = False, keep_final: bool = True,
                        keep_updates: bool = False) -> dict:
        """Output buffers of an ``n_steps`` rollout.  Uninitialised: the kernel writes every
        element of every buffer it is given (all ``n_alloc`` envs, all steps), and ``rollout``
        writes the flip masks itself when it does not draw them.  Allocate them before a
        hipGraph capture so that the graph holds the rollout launch alone.  ``keep_updates``:
        the synchronous updates of every env-step (uint16; the settle length under the settle law)."""
        W, n, dev = self.words, self.n_alloc, self.device
        return {"_n_steps": n_steps,
                "flipmask": torch.empty(n_steps, W, n, dtype=torch.int32, device=dev),
                "reward": torch.empty(n_steps, n, dtype=torch.float32, device=dev),
                "flags": torch.empty(n_steps, n, dtype=torch.uint8, device=dev),
                "obs": torch.empty(n_steps, W, n, dtype=torch.int32, device=dev) if keep_obs else None,
                "final_state": torch.empty(n_steps, W, n, dtype=torch.int32, device=dev) if keep_final else None,
                "updates": torch.empty(n_steps, n, dtype=torch.int16, device=dev) if keep_updates else None}

    def rollout(self, n_steps: int, flipmasks: Optional[torch.Tensor] = None, random_actions: bool = True,
                keep_obs: bool = False, keep_final: bool = True, out: Optional[dict] = None,
                keep_updates: bool = False, copy: Optional[tuple] = None) -> dict:
        """``n_steps`` env steps in one ``pbn_rollout_ex`` launch (state kept on chip).

        flipmasks: optional (n_steps, W, num_envs) interventions (else in-kernel random
        actions when ``random_actions``, else none).  Returns views of
        ``flipmask`` / ``reward`` / ``flags`` (+ ``obs`` / ``final_state`` / ``updates``) shaped
        (n_steps, ...); pass ``out`` (a previous result) to reuse its buffers.
        ``copy = (dst, src)``: two contiguous device buffers of equal size (16-byte multiples, not
        this launch's outputs); dst <- src rides along the launch (``pbn_rollout_copy``, done when
        the launch is)."""
        L = _lib.load()
        n, k = self.n_alloc, self.num_envs
        if out is None or out["_n_steps"] != n_steps:
            out = self.rollout_buffers(n_steps, keep_obs, keep_final, keep_updates)
        mode = _lib.MODE_AUTORESET if self.autoreset else 0
        if flipmasks is not None:
            out["flipmask"][:, :, :k].copy_(flipmasks)
            out["flipmask"][:, :, k:].zero_()
        elif random_actions:
            mode |= _lib.MODE_RANDOM_ACTIONS
        else:
            out["flipmask"].zero_()
        ptr = lambda t: t.data_ptr() if t is not None else None  # noqa: E731
        with torch.cuda.device(self.device):
            if copy is not None:
                dst, src = copy
                if dst.numel() * dst.element_size() != src.numel() * src.element_size():
                    raise ValueError("copy: dst and src differ in size")
                if not (dst.is_contiguous() and src.is_contiguous()) or dst.device != src.device or \
                        src.device.type != "cuda":
                    raise ValueError("copy: dst and src must be contiguous tensors on the env's GPU")
                # the launch writes its outputs and the env's state, t and target while the copy
                # reads src and writes dst: neither range may overlap them (the kernel cannot check)
                own = [t for t in (self.state, self.target, self.t, *(v for key, v in out.items()
                                                                      if key != "_n_steps"))
                       if isinstance(t, torch.Tensor)]
                for name, c in (("dst", dst), ("src", src)):
                    lo, hi = c.data_ptr(), c.data_ptr() + c.numel() * c.element_size()
                    for t in own:
                        t_lo = t.data_ptr()
                        if lo < t_lo + t.numel() * t.element_size() and t_lo < hi:
                            raise ValueError(f"copy: {name} overlaps a buffer this launch writes")
                _lib.check(L.pbn_rollout_copy(self.net.handle, self.seed, self.step_index, self.env_offset, n,
                                              n_steps, mode, self.state.data_ptr(), out["flipmask"].data_ptr(),
                                              self.target.data_ptr(), self.t.data_ptr(), ptr(out["obs"]),
                                              ptr(out["final_state"]), out["reward"].data_ptr(),
                                              out["flags"].data_ptr(), ptr(out.get("updates")), dst.data_ptr(),
                                              src.data_ptr(), src.numel() * src.element_size(), self._stream()),
                           "pbn_rollout_copy")
            else:
                _lib.check(L.pbn_rollout_ex(self.net.handle, self.seed, self.step_index, self.env_offset, n,
                                            n_steps, mode, self.state.data_ptr(), out["flipmask"].data_ptr(),
                                            self.target.data_ptr(), self.t.data_ptr(), ptr(out["obs"]),
                                            ptr(out["final_state"]), out["reward"].data_ptr(),
                                            out["flags"].data_ptr(), ptr(out.get("updates")), self._stream()),
                           "pbn_rollout_ex")
        self.step_index += n_steps
        return out

    def step(self, actions: Optional[torch.Tensor] = None):
        """gymnasium-vector style: actions (n, k) in [0, N] (or None = no intervention).
        Returns (state_words, reward, terminated, truncated, info)."""
        fm = None if actions is None else actions_to_flipmask(actions.to(self.device), self.n_nodes)
        state, reward, flags = self.step_flipmask(fm)
        terminated = (flags & _lib.FLAG_TERMINATED) != 0
        truncated = (flags & _lib.FLAG_TRUNCATED) != 0
        info = {"flags": flags}
        if self.final_state is not None:
            info["final_state"] = self.final_state[:, : self.num_envs]
        return state, reward, terminated, truncated, info

    def set_state(self, words: torch.Tensor, target: Optional[torch.Tensor] = None,
                  t: Optional[torch.Tensor] = None) -> None:
        self.state[:, : self.num_envs].copy_(words)
        if target is not None:
            self.target[: self.num_envs].copy_(target)
        if t is not None:
            self.t[: self.num_envs].copy_(t)

    def set_spec(self, spec: EnvSpec) -> None:
        """Swap in a spec of the same network shape (e.g. a grown attractor set): the device
        tables are rebuilt; state, targets and step counter are kept."""
        if spec.n != self.n_nodes or spec.words != self.words:
            raise ValueError("set_spec needs a spec with the same node count")
        with torch.cuda.device(self.device):
            net = _lib.NetHandle(spec)
        self.net.close()
        self.net, self.spec = net, spec

    def close(self) -> None:
        self.net.close()
