"""Batched BDQ frame loop on the GPU.

The reference steps one env per frame: ``BranchingDQN.predict`` stacks (state, target) on the
host into a float (2, 1, N) tensor, runs ``BranchingQNetwork``, takes argmax over each of the
3 action branches (bdq_model/__init__.py:69-98), and ``env.step(list(action.unique()))``
flips node a-1 for every action a > 0 (:81-84,176-177).  Here one frame covers a whole
``VectorPBNEnv`` batch, and nothing leaves HBM (BatchedBDQ.step):

    pbn_bilinear_targets   packed state + target id -> the bilinear layer (+ LeakyReLU)   (HIP)
    pbn_qnet_heads         the rest of the network -> raw head outputs (4, n, N+1)         (HIP, MFMA)
    pbn_heads_to_flipmask  dueling combination + epsilon-greedy -> flip-mask words (W, n)  (HIP)
    pbn_qnet_flipmask      the two above in one launch                                    (HIP)
    pbn_qnet_flipmask_from_state  all of it from the packed state, one launch (act_q, step) (HIP, MFMA)
    pbn_step               the PBN transition                                             (HIP)

(``fused_tail=False`` runs the layers after the bilinear one in PyTorch instead.)

``BranchingQNetwork`` keeps the reference module tree (bdq_model/network.py:24-63), so the
reference's checkpoints load into it with ``load_state_dict``; its own forward (used for
training) computes the bilinear layer as GEMMs (MyBilinear), and ``pbn_obs_unpack`` +
``pbn_q_to_flipmask`` give the unfused path on an explicit observation and Q.
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _lib
from .vector_env import VectorPBNEnv

__all__ = ["MyBilinear", "BranchingQNetwork", "BatchedBDQ", "load_bdq_checkpoint", "formula_weights"]


class MyBilinear(nn.Module):
    """nn.Bilinear over input[0], input[1] (bdq_model/network.py:8-21), as GEMMs.

    y[b, o] = bias[o] + sum_ij a[b, i] W[o, i, j] b[b, j] is evaluated in one of two orders:
      outer     (B, N1*N2) @ (N1*N2, out): one GEMM over the outer product (large batches:
                the acting forward over all envs)
      contract  T = b @ W.view(out*N1, N2)^T, then y = T.view(B, out, N1) @ a (batched): for
                small batches (replay updates), where the outer form's (B x out) output is one
                or two GEMM tiles and leaves the chip idle
    ``form`` = "auto" picks contract below ``contract_rows`` rows."""

    contract_rows = 4096

    def __init__(self, input1_dim: int, input2_dim: int, output_dim: int):
        super().__init__()
        self.input1_dim, self.input2_dim, self.output_dim = input1_dim, input2_dim, output_dim
        self.bilinear = nn.Bilinear(input1_dim, input2_dim, output_dim)
        self.form = "auto"

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        a, b = x[0], x[1]
        lead = a.shape[:-1]
        a2 = a.reshape(-1, self.input1_dim)
        b2 = b.reshape(-1, self.input2_dim)
        rows = a2.shape[0]
        form = self.form if self.form != "auto" else ("contract" if rows < self.contract_rows else "outer")
        if form == "contract":
            t = b2 @ self.bilinear.weight.reshape(-1, self.input2_dim).t()          # (B, out*N1)
            y = torch.baddbmm(self.bilinear.bias.view(1, -1, 1), t.view(rows, self.output_dim, self.input1_dim),
                              a2.unsqueeze(2)).squeeze(2)
        else:
            outer = (a2[:, :, None] * b2[:, None, :]).reshape(rows, -1)
            w = self.bilinear.weight.reshape(self.output_dim, -1)
            y = torch.addmm(self.bilinear.bias, outer, w.t())
        return y.reshape(*lead, self.output_dim)

    def target_table(self, targets: torch.Tensor) -> torch.Tensor:
        """T[a, i, o] = sum_j targets[a, j] W[o, i, j] for (A, N2) 0/1 target rows: the layer
        contracted with each target, the table pbn_bilinear_targets reads."""
        w = self.bilinear.weight                                     # (out, N1, N2)
        t = targets.to(w.dtype) @ w.permute(2, 1, 0).reshape(self.input2_dim, -1)
        return t.view(targets.shape[0], self.input1_dim, self.output_dim)


def _mlp(i: int, h: int, o: int) -> nn.Sequential:
    return nn.Sequential(nn.Linear(i, h), nn.LeakyReLU(), nn.Linear(h, o))


class BranchingQNetwork(nn.Module):
    """Dueling branching Q-network of bdq_model/network.py:24-63, same parameter names.

    observation = (N, N) (state and target lengths), action_space_dimension = N + 1,
    number_of_actions = branches (3 in train_BDQ.py:83).  forward: (2, B, N) -> (B, K, N+1),
    q = value + advantage - mean(advantage) per branch (:59-61)."""

    def __init__(self, observation: Tuple[int, int], action_space_dimension: int, number_of_actions: int):
        super().__init__()
        self.ac_dim = action_space_dimension
        self.n = number_of_actions
        s, t = observation
        self.model = nn.Sequential(MyBilinear(s, t, 256), nn.LeakyReLU(),
                                   nn.Linear(256, 128), nn.LeakyReLU(),
                                   nn.Linear(128, 64), nn.LeakyReLU(),
                                   nn.Linear(64, 32), nn.LeakyReLU())
        self.value_head = _mlp(32, 64, 1)
        self.adv_heads = nn.ModuleList([_mlp(32, 64, action_space_dimension) for _ in range(number_of_actions)])

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self.forward_tail(self.model[0](x))

    def forward_tail(self, y: torch.Tensor, skip_act: bool = False) -> torch.Tensor:
        """The network after the bilinear layer: y (B, 256) -> Q (B, K, A); ``skip_act``: y
        already went through model[1] (the LeakyReLU)."""
        return self.dueling(self.forward_heads(y, skip_act))

    @staticmethod
    def dueling(out: torch.Tensor) -> torch.Tensor:
        """Raw head outputs (K+1, B, A) -> Q (B, K, A) = v + adv - mean(adv) (:59-61)."""
        v = out[0, :, :1]                                             # (B, 1)
        adv = out[1:].transpose(0, 1)                                 # (B, K, A)
        return v.unsqueeze(2) + adv - adv.mean(2, keepdim=True)

    def head_weights(self):
        """(w1, b1, w2, b2): the value head and the K advantage heads as one (32 -> 64(K+1))
        layer and one batched (K+1) x (64 -> A) layer; the value head is zero-padded to A
        outputs (only output 0 is used)."""
        heads = [self.value_head] + list(self.adv_heads)
        A = self.ac_dim
        w1 = torch.cat([hd[0].weight for hd in heads], 0)             # (64(K+1), 32)
        b1 = torch.cat([hd[0].bias for hd in heads], 0)
        w2 = torch.stack([F.pad(self.value_head[2].weight, (0, 0, 0, A - 1))]
                         + [hd[2].weight for hd in self.adv_heads])   # (K+1, A, 64)
        b2 = torch.stack([F.pad(self.value_head[2].bias, (0, A - 1))]
                         + [hd[2].bias for hd in self.adv_heads]).unsqueeze(1)   # (K+1, 1, A)
        return w1, b1, w2, b2

    def forward_heads(self, y: torch.Tensor, skip_act: bool = False, weights=None) -> torch.Tensor:
        """y (B, 256) -> the raw outputs (K+1, B, A) of the value head (output 0) and the
        advantage heads, before the dueling combination.  ``weights``: head_weights() computed
        beforehand (prepacked for a frozen network)."""
        h = self.model[2:](y) if skip_act else self.model[1:](y)      # (B, 32)
        # the value head and the K advantage heads read the same h: their first layers run as
        # one (32 -> 64(K+1)) GEMM, their second layers as one batched GEMM over K+1 heads
        w1, b1, w2, b2 = weights if weights is not None else self.head_weights()
        z = F.leaky_relu(torch.addmm(b1, h, w1.t()))                  # (B, 64(K+1))
        z = z.view(z.shape[0], w2.shape[0], -1).transpose(0, 1)       # (K+1, B, 64)
        return torch.baddbmm(b2, z, w2.transpose(1, 2))               # (K+1, B, A)


class BatchedBDQ:
    """The BDQ acting loop over a VectorPBNEnv: obs unpack -> Q -> epsilon-greedy flip masks ->
    pbn_step, all on the env's device and the current stream (graph-capturable)."""

    def __init__(self, env: VectorPBNEnv, qnet: Optional[BranchingQNetwork] = None, *, branches: int = 3,
                 epsilon: float = 0.0, fused_tail: bool = True):
        self.env = env
        N = env.n_nodes
        self.branches = int(branches)
        self.q = qnet if qnet is not None else BranchingQNetwork((N, N), N + 1, self.branches)
        self.q = self.q.to(env.device).eval()
        self.epsilon = float(epsilon)
        n = env.n_alloc
        self.obs = torch.empty(2, n, N, dtype=torch.float32, device=env.device)
        self.actions = torch.empty(n, self.branches, dtype=torch.int32, device=env.device)
        # first state of every attractor: the target half of the observation (pbn_obs_unpack)
        atts = env.spec.attractors
        self.targets = torch.tensor([list(a[0]) for a in atts], dtype=torch.float32,
                                    device=env.device).reshape(len(atts), N)
        self.fast = isinstance(self.q.model[0], MyBilinear)
        act = self.q.model[1] if len(self.q.model) > 1 else None
        self._act = isinstance(act, nn.LeakyReLU)
        self._slope = float(act.negative_slope) if self._act else 0.0
        self._pack, self._pack_key = None, None
        # set by a learner that keeps the weight-derived operands itself (FusedBDQUpdate.acting_pack)
        self.pack_provider = None
        self._y = torch.empty(n, self.q.model[0].output_dim if self.fast else 1, dtype=torch.float32,
                              device=env.device)
        self.fused_tail = bool(fused_tail) and self._tail_fusable()
        self._heads = (torch.empty(self.branches + 1, n, env.n_nodes + 1, dtype=torch.float32, device=env.device)
                       if self.fused_tail else None)

    def _tail_fusable(self) -> bool:
        """pbn_qnet_heads implements exactly BranchingQNetwork's layers after the bilinear one
        (256-128-64-32 trunk, 32-64-A heads, one LeakyReLU slope)."""
        m = self.q.model
        if not (self.fast and self._act and len(m) == 8 and m[0].output_dim == 256):
            return False
        dims = [(m[2], 256, 128), (m[4], 128, 64), (m[6], 64, 32)]
        if any(not isinstance(l, nn.Linear) or (l.in_features, l.out_features) != (i, o) for l, i, o in dims):
            return False
        acts = [m[1], m[3], m[5], m[7], self.q.value_head[1]] + [hd[1] for hd in self.q.adv_heads]
        if any(not isinstance(a, nn.LeakyReLU) or float(a.negative_slope) != self._slope for a in acts):
            return False
        return self.q.n == self.branches and self.branches + 1 <= 8 and self.q.ac_dim <= 128

    def observe(self) -> torch.Tensor:
        """(2, n, N) fp32: env states and their target attractors' first states."""
        env = self.env
        L = _lib.load()
        with torch.cuda.device(env.device):
            _lib.check(L.pbn_obs_unpack(env.net.handle, env.n_alloc, env.state.data_ptr(), env.target.data_ptr(),
                                        self.obs.data_ptr(), env._stream()), "pbn_obs_unpack")
        return self.obs

    def act(self, q: torch.Tensor, epsilon: Optional[float] = None) -> torch.Tensor:
        """Q (n, K, N+1) -> env.flipmask (W, n) and self.actions (n, K), keyed by the env's
        next step index."""
        env = self.env
        q = q.contiguous()
        if q.shape != (env.n_alloc, self.branches, env.n_nodes + 1):
            raise ValueError(f"Q must have shape {(env.n_alloc, self.branches, env.n_nodes + 1)}")
        eps = self.epsilon if epsilon is None else float(epsilon)
        L = _lib.load()
        with torch.cuda.device(env.device):
            _lib.check(L.pbn_q_to_flipmask(env.net.handle, env.seed, env.step_index, env.env_offset, env.n_alloc,
                                           self.branches, env.n_nodes + 1, q.data_ptr(), eps,
                                           env.flipmask.data_ptr(), self.actions.data_ptr(), env._stream()),
                       "pbn_q_to_flipmask")
        return env.flipmask

    def act_dev(self, q: torch.Tensor, step_t: torch.Tensor, epsilon_t: Optional[torch.Tensor] = None,
                epsilon: Optional[float] = None) -> torch.Tensor:
        """``act`` through ``pbn_q_to_flipmask_dev``: the step index (int64) and, when given,
        epsilon (float32) are read from one-element device tensors (graph replays)."""
        env = self.env
        q = q.contiguous()
        if q.shape != (env.n_alloc, self.branches, env.n_nodes + 1):
            raise ValueError(f"Q must have shape {(env.n_alloc, self.branches, env.n_nodes + 1)}")
        if step_t.dtype != torch.int64 or step_t.numel() != 1:
            raise ValueError("step_t must be a one-element int64 tensor")
        if epsilon_t is not None and (epsilon_t.dtype != torch.float32 or epsilon_t.numel() != 1):
            raise ValueError("epsilon_t must be a one-element float32 tensor")
        eps = self.epsilon if epsilon is None else float(epsilon)
        L = _lib.load()
        with torch.cuda.device(env.device):
            _lib.check(L.pbn_q_to_flipmask_dev(env.net.handle, env.seed, step_t.data_ptr(), env.env_offset,
                                               env.n_alloc, self.branches, env.n_nodes + 1, q.data_ptr(), eps,
                                               epsilon_t.data_ptr() if epsilon_t is not None else None,
                                               env.flipmask.data_ptr(), self.actions.data_ptr(), env._stream()),
                       "pbn_q_to_flipmask_dev")
        return env.flipmask

    def q_heads(self) -> torch.Tensor:
        """The raw head outputs (K+1, n, A) of every env's observation (q_values before the
        dueling combination, which pbn_heads_to_flipmask does)."""
        return self._forward(heads=True)

    def q_values(self) -> torch.Tensor:
        """Q (n, K, N+1) of every env's (state, target) observation.  With the reference's
        MyBilinear first layer this skips the fp32 observation: pbn_bilinear_targets computes
        the bilinear layer from the packed state and a per-target table (one small GEMM), and
        the rest of the network runs in PyTorch.  Equal to ``q(observe())`` up to fp32
        summation order."""
        return self._forward(heads=False)

    def _packed(self):
        """Weight-derived operands of the fast forward: the target table of the bilinear layer,
        its bias and the head weights.  For a network in eval mode they are computed once per
        version of its parameters (prepacked, as inference packs weights at load time) and
        reused, so a frame runs no assembly kernels; a captured frame keeps the pack of its
        capture (re-capture after changing the weights).  In train mode (the learner) they are
        recomputed every call."""
        if self.pack_provider is not None:
            return self.pack_provider()
        key = None
        if not self.q.training:
            key = tuple((p.data_ptr(), p._version) for p in self.q.parameters())
            if key == self._pack_key:
                return self._pack
        bil = self.q.model[0]
        T = bil.target_table(self.targets).contiguous() if self.targets.shape[0] else None
        # the fused kernels' layout of the same table: [a][i][j][q] = T[a][i][16 q + j]
        Tq = T.view(T.shape[0], T.shape[1], 16, 16).transpose(2, 3).contiguous() if T is not None else None
        pack = (T, bil.bilinear.bias.contiguous(), self.q.head_weights(), Tq)
        if key is not None:
            self._pack, self._pack_key = pack, key
        return pack

    def bilinear(self):
        """One ``pbn_bilinear_targets`` launch into ``self._y`` (the first layer + LeakyReLU of the
        fast forward); returns the head weights of the same pack."""
        env = self.env
        bil = self.q.model[0]
        T, bias, hw, Tq = self._packed()
        if T is None and Tq is not None:   # (a provider's pack holds only the fused layout)
            T = Tq.transpose(2, 3).reshape(Tq.shape[0], Tq.shape[1], -1).contiguous()
        L = _lib.load()
        with torch.cuda.device(env.device):
            _lib.check(L.pbn_bilinear_targets(env.net.handle, env.n_alloc, env.state.data_ptr(),
                                              env.target.data_ptr(), T.data_ptr() if T is not None else None,
                                              bias.data_ptr(), bil.output_dim, 1 if self._act else 0,
                                              self._slope, self._y.data_ptr(), env._stream()),
                       "pbn_bilinear_targets")
        return hw

    def _forward(self, heads: bool) -> torch.Tensor:
        if not self.fast:
            y = self.q.model[0](self.observe())
            return self.q.forward_heads(y) if heads else self.q.forward_tail(y)
        if self.fused_tail and not (torch.is_grad_enabled() and self.q.training):   # (no autograd through it)
            out = self._tail_kernel()
        else:
            hw = self.bilinear()
            # the kernel applied model[1] (LeakyReLU) when _act
            out = self.q.forward_heads(self._y, skip_act=self._act, weights=hw)
        return out if heads else self.q.dueling(out)

    def _tail_operands(self):
        """Device pointers of the fused kernels' operands after the state: the bilinear layer's
        target table and bias, then the trunk and the stacked head weights."""
        m = self.q.model
        _, bias, (w1, b1, w2, b2), T = self._packed()
        ts = [bias, m[2].weight, m[2].bias, m[4].weight, m[4].bias, m[6].weight, m[6].bias, w1, b1, w2, b2]
        ts = [t.detach().contiguous() for t in ts]
        return [T.data_ptr() if T is not None else None] + [t.data_ptr() for t in ts], ts

    def _tail_kernel(self) -> torch.Tensor:
        """pbn_qnet_heads_from_state: the whole network from the packed state -> self._heads
        (K+1, n, A), one launch."""
        env = self.env
        ptrs, _keep = self._tail_operands()
        L = _lib.load()
        with torch.cuda.device(env.device):
            _lib.check(L.pbn_qnet_heads_from_state(env.net.handle, env.n_alloc, env.state.data_ptr(),
                                                   env.target.data_ptr(), *ptrs, self.branches + 1,
                                                   env.n_nodes + 1, self._slope, self._heads.data_ptr(),
                                                   env._stream()), "pbn_qnet_heads_from_state")
        return self._heads

    def act_heads(self, heads: torch.Tensor, epsilon: Optional[float] = None,
                  step_t: Optional[torch.Tensor] = None, epsilon_t: Optional[torch.Tensor] = None) -> torch.Tensor:
        """``act`` on raw head outputs (K+1, n, N+1): pbn_heads_to_flipmask does the dueling
        combination, epsilon-greedy and flip masks in one launch.  ``step_t`` / ``epsilon_t``:
        optional one-element device tensors (int64 / float32) read when the kernel runs."""
        env = self.env
        heads = heads.contiguous()
        if heads.shape != (self.branches + 1, env.n_alloc, env.n_nodes + 1):
            raise ValueError(f"heads must have shape {(self.branches + 1, env.n_alloc, env.n_nodes + 1)}")
        eps = self.epsilon if epsilon is None else float(epsilon)
        L = _lib.load()
        with torch.cuda.device(env.device):
            _lib.check(L.pbn_heads_to_flipmask(env.net.handle, env.seed, env.step_index,
                                               step_t.data_ptr() if step_t is not None else None,
                                               env.env_offset, env.n_alloc, self.branches, env.n_nodes + 1,
                                               heads.data_ptr(), eps,
                                               epsilon_t.data_ptr() if epsilon_t is not None else None,
                                               env.flipmask.data_ptr(), self.actions.data_ptr(), env._stream()),
                       "pbn_heads_to_flipmask")
        return env.flipmask

    @torch.no_grad()
    def act_q(self, epsilon: Optional[float] = None, step_t: Optional[torch.Tensor] = None,
              epsilon_t: Optional[torch.Tensor] = None) -> torch.Tensor:
        """``predict`` + epsilon-greedy for every env (bdq_model/__init__.py:69-98): Q of the
        current observations -> env.flipmask and self.actions.  With the fused tail this is one
        launch, pbn_qnet_flipmask_from_state (the whole network from the packed state, no
        activations in HBM), else q_heads() + act_heads().  ``step_t`` / ``epsilon_t`` as act_heads."""
        if not (self.fast and self.fused_tail):
            return self.act_heads(self.q_heads(), epsilon, step_t=step_t, epsilon_t=epsilon_t)
        if step_t is not None and (step_t.dtype != torch.int64 or step_t.numel() != 1):
            raise ValueError("step_t must be a one-element int64 tensor")
        if epsilon_t is not None and (epsilon_t.dtype != torch.float32 or epsilon_t.numel() != 1):
            raise ValueError("epsilon_t must be a one-element float32 tensor")
        env = self.env
        ptrs, _keep = self._tail_operands()
        eps = self.epsilon if epsilon is None else float(epsilon)
        L = _lib.load()
        with torch.cuda.device(env.device):
            _lib.check(L.pbn_qnet_flipmask_from_state(env.net.handle, env.seed, env.step_index,
                                                      step_t.data_ptr() if step_t is not None else None,
                                                      env.env_offset, env.n_alloc, env.state.data_ptr(),
                                                      env.target.data_ptr(), *ptrs, self.branches, env.n_nodes + 1,
                                                      self._slope, eps,
                                                      epsilon_t.data_ptr() if epsilon_t is not None else None,
                                                      env.flipmask.data_ptr(), self.actions.data_ptr(),
                                                      env._stream()),
                       "pbn_qnet_flipmask_from_state")
        return env.flipmask

    @torch.no_grad()
    def step(self, epsilon: Optional[float] = None):
        """One frame for every env; returns (state', reward, flags) views as VectorPBNEnv.step_flipmask."""
        self.act_q(epsilon)
        return self.env.step_flipmask(use_current=True)


def load_bdq_checkpoint(qnet: BranchingQNetwork, path: str, prefix: str = "q.") -> BranchingQNetwork:
    """Load the ``q`` (or ``target``) network of a reference BranchingDQN checkpoint
    (``torch.save(self.state_dict())`` at bdq_model/__init__.py:237,240-244) into ``qnet``.
    Tensors only (``weights_only=True``); nothing in the file is executed."""
    sd = torch.load(path, map_location="cpu", weights_only=True)
    sub = {k[len(prefix):]: v for k, v in sd.items() if k.startswith(prefix)}
    if not sub:
        sub = dict(sd)
    qnet.load_state_dict(sub)
    return qnet


@torch.no_grad()
def formula_weights(qnet: nn.Module) -> nn.Module:
    """Deterministic, RNG-free parameters (sin ramps scaled by 1/sqrt(fan-in)) for golden
    vectors that must not depend on torch's generator across versions."""
    for idx, (name, p) in enumerate(sorted(qnet.named_parameters())):
        k = torch.arange(p.numel(), dtype=torch.float64)
        fan_in = p.shape[-1] if p.dim() >= 2 else max(1, p.numel())
        vals = torch.sin(0.731 * k + 0.5 * idx) / (fan_in ** 0.5)
        p.copy_(vals.reshape(p.shape).to(p.dtype))
    return qnet
