"""On-device replay and the BDQ learner update (rows A9, A10).

The reference keeps transitions as host ``Transition`` namedtuples in a Python list
(``ExperienceReplay``, bdq_model/memory.py:17-62), and every update ``np.stack``s 256 of them
and copies them to the GPU (``update_policy``, bdq_model/__init__.py:100-109).  Here the
replay is a ring of packed transitions in HBM, filled straight from the batched env:

    state, next_state   int32 [W][capacity]   packed words (bit i of word w = node 32w + i)
    target              uint8 [capacity]      target attractor id
    action              int32 [capacity][K]   the branch actions
    reward              float32 [capacity]
    done                uint8 [capacity]      terminated or truncated

Sampling gathers rows by index and unpacks them to the fp32 (2, B, N) network input with
``pbn_obs_unpack`` (the HIP kernel the acting frame uses), so nothing goes through the host.
Indices are drawn with replacement (torch's device generator); ``random.sample`` at
bdq_model/memory.py:62 draws without replacement, which only matters for batches comparable
to the ring size.

``bdq_update`` restates ``update_policy`` (bdq_model/__init__.py:100-139) on such a batch:
double-DQN targets ``r + gamma * mask * Q_target(s', argmax_a Q(s', a))`` with the
reference's ``mask = done`` (:109,122 -- it bootstraps only on done transitions; kept as is),
MSE loss, gradients clamped to [-1, 1] (:129-130), one Adam step, and every
``target_update`` updates the target network moves halfway to the online one (:133-139).
"""
from __future__ import annotations

import ctypes
from typing import Dict, List, Optional

import torch
import torch.nn.functional as F

from . import _lib
from .agent import BatchedBDQ, BranchingQNetwork
from .vector_env import VectorPBNEnv

__all__ = ["DeviceReplay", "bdq_update", "soft_update", "BDQLearner", "FusedBDQUpdate", "bdq_layout",
           "fused_update_supported"]


class DeviceReplay:
    def __init__(self, capacity: int, words: int, branches: int, device):
        self.capacity = int(capacity)
        self.words = int(words)
        self.device = torch.device(device)
        dev = self.device
        self.state = torch.zeros(words, capacity, dtype=torch.int32, device=dev)
        self.next_state = torch.zeros(words, capacity, dtype=torch.int32, device=dev)
        self.target = torch.zeros(capacity, dtype=torch.uint8, device=dev)
        self.action = torch.zeros(capacity, branches, dtype=torch.int32, device=dev)
        self.reward = torch.zeros(capacity, dtype=torch.float32, device=dev)
        self.done = torch.zeros(capacity, dtype=torch.uint8, device=dev)
        self.pos = 0
        self.size = 0

    def _slots(self, n: int) -> torch.Tensor:
        return (torch.arange(n, device=self.device, dtype=torch.int64) + self.pos) % self.capacity

    def store(self, state: torch.Tensor, target: torch.Tensor, action: torch.Tensor, reward: torch.Tensor,
              next_state: torch.Tensor, done: torch.Tensor) -> None:
        """Append n transitions: state / next_state (W, n) words, target (n,), action (n, K),
        reward (n,), done (n,) (any dtype castable to the ring's)."""
        n = target.shape[0]
        if n > self.capacity:
            raise ValueError("more transitions than the ring holds")
        idx = self._slots(n)
        self.state.index_copy_(1, idx, state)
        self.next_state.index_copy_(1, idx, next_state)
        self.target.index_copy_(0, idx, target.to(torch.uint8))
        self.action.index_copy_(0, idx, action.to(torch.int32))
        self.reward.index_copy_(0, idx, reward.to(torch.float32))
        self.done.index_copy_(0, idx, done.to(torch.uint8))
        self.pos = (self.pos + n) % self.capacity
        self.size = min(self.size + n, self.capacity)

    def store_at(self, pos_t: torch.Tensor, size_t: torch.Tensor, state, target, action, reward, next_state,
                 done, *, done_mask: int = 0, done_out: Optional[torch.Tensor] = None, advance: bool = True,
                 state_copy=None, target_copy=None) -> None:
        """``store`` with the ring position and fill level held in one-element int64 device
        tensors (advanced here, on the stream, unless ``advance`` is False) instead of host ints:
        graph-capturable.  The caller mirrors them in ``pos`` / ``size``.  ``done_mask`` != 0:
        ``done`` is the env's flags and a transition is done when ``flags & done_mask``;
        ``done_out`` (uint8 [n]) then receives those 0/1 values too.  ``state_copy`` / ``target_copy``:
        optional (dst, src) pairs copied element by element in the same pass, after the element of
        ``state`` / ``target`` is read (dst may be ``state`` / ``target`` itself; GPU path only)."""
        n = target.shape[0]
        if n > self.capacity:
            raise ValueError("more transitions than the ring holds")
        if (self.device.type == "cuda" and state.dtype == torch.int32 and next_state.dtype == torch.int32
                and target.dtype == torch.uint8 and action.dtype == torch.int32 and reward.dtype == torch.float32
                and done.dtype in (torch.bool, torch.uint8)):
            # the six field copies in one launch (pbn_replay_store)
            st, nst, act = state.contiguous(), next_state.contiguous(), action.contiguous()
            if done_out is not None and (done_out.dtype != torch.uint8 or done_out.numel() < n):
                raise ValueError("done_out must be uint8 with n elements")
            L = _lib.load()
            with torch.cuda.device(self.device):
                _lib.check(L.pbn_replay_store(n, pos_t.data_ptr(), self.capacity, self.words, self.action.shape[1],
                                              st.data_ptr(), nst.data_ptr(), target.contiguous().data_ptr(),
                                              act.data_ptr(), reward.contiguous().data_ptr(),
                                              done.contiguous().data_ptr(), int(done_mask),
                                              done_out.data_ptr() if done_out is not None else None,
                                              self.state.data_ptr(), self.next_state.data_ptr(), self.target.data_ptr(),
                                              self.action.data_ptr(), self.reward.data_ptr(), self.done.data_ptr(),
                                              *(t.data_ptr() if t is not None else None
                                                for t in (state_copy or (None, None)) + (target_copy or (None, None))),
                                              torch.cuda.current_stream(self.device).cuda_stream), "pbn_replay_store")
            if advance:
                pos_t.add_(n).remainder_(self.capacity)
                size_t.add_(n).clamp_(max=self.capacity)
            return
        if state_copy is not None or target_copy is not None:
            raise ValueError("state_copy / target_copy need the GPU path (int32 / uint8 / float32 fields)")
        if done_mask:
            done = (done & done_mask) != 0
            if done_out is not None:
                done_out[:n].copy_(done)
        idx = (torch.arange(n, device=self.device, dtype=torch.int64) + pos_t) % self.capacity
        self.state.index_copy_(1, idx, state)
        self.next_state.index_copy_(1, idx, next_state)
        self.target.index_copy_(0, idx, target.to(torch.uint8))
        self.action.index_copy_(0, idx, action.to(torch.int32))
        self.reward.index_copy_(0, idx, reward.to(torch.float32))
        self.done.index_copy_(0, idx, done.to(torch.uint8))
        if advance:
            pos_t.add_(n).remainder_(self.capacity)
            size_t.add_(n).clamp_(max=self.capacity)

    def sample_indices(self, batch: int, generator: Optional[torch.Generator] = None,
                       size_t: Optional[torch.Tensor] = None) -> torch.Tensor:
        """``batch`` indices uniform over the filled part, with replacement: floor(u * size)
        for fp64 uniforms u.  ``size_t`` (a one-element int64 device tensor) replaces the host
        fill level in graph-captured frames; both forms draw the same indices."""
        if size_t is None:
            if self.size == 0:
                raise ValueError("empty replay")
            size_t = torch.full((1,), self.size, dtype=torch.int64, device=self.device)
        u = torch.rand(batch, dtype=torch.float64, device=self.device, generator=generator)
        idx = (u * size_t).long()
        return torch.minimum(idx, size_t - 1)

    def sample_rows(self, idx_out: torch.Tensor, seed: int, counter_t: torch.Tensor, size_t: torch.Tensor) -> torch.Tensor:
        """Fill ``idx_out`` (int64) with rows uniform over [0, size) with replacement, from the
        Philox REPLAY stream of (seed, row, *counter_t) (pbn_replay_advance; counter_t advances):
        one launch, graph-capturable, and the same rows eager or captured."""
        L = _lib.load()
        with torch.cuda.device(self.device):
            _lib.check(L.pbn_replay_advance(0, self.capacity, None, size_t.data_ptr(), None, None, None, 0.0, 0.0,
                                            idx_out.numel(), seed, counter_t.data_ptr(), idx_out.data_ptr(),
                                            torch.cuda.current_stream(self.device).cuda_stream), "pbn_replay_advance")
        return idx_out

    def gather(self, idx: torch.Tensor, net_handle, stream=None) -> Dict[str, torch.Tensor]:
        """Rows ``idx`` (B a multiple of 32) as network inputs, in one launch (``pbn_replay_batch``):
        x fp32 (2, 2B, N) = obs and next_obs concatenated by rows (obs / next_obs are its halves:
        state or next state, and the target attractor's first state), actions (B, K, 1) int64,
        rewards (B, 1), masks (B, 1)."""
        B = idx.shape[0]
        if B % 32:
            raise ValueError("batch size must be a multiple of 32")
        N = net_handle.spec.n
        K = self.action.shape[1]
        dev = self.device
        x = torch.empty(2, 2 * B, N, dtype=torch.float32, device=dev)
        actions = torch.empty(B, K, dtype=torch.int64, device=dev)
        rewards = torch.empty(B, dtype=torch.float32, device=dev)
        masks = torch.empty(B, dtype=torch.float32, device=dev)
        idx = idx.to(torch.int64).contiguous()
        L = _lib.load()
        s = stream if stream is not None else torch.cuda.current_stream(dev).cuda_stream
        with torch.cuda.device(dev):
            _lib.check(L.pbn_replay_batch(net_handle.handle, B, idx.data_ptr(), self.capacity, self.state.data_ptr(),
                                          self.next_state.data_ptr(), self.target.data_ptr(), self.action.data_ptr(),
                                          K, self.reward.data_ptr(), self.done.data_ptr(), x.data_ptr(),
                                          actions.data_ptr(), rewards.data_ptr(), masks.data_ptr(), s),
                       "pbn_replay_batch")
        return {"x": x, "obs": x[:, :B], "next_obs": x[:, B:], "actions": actions.unsqueeze(-1),
                "rewards": rewards.reshape(-1, 1), "masks": masks.reshape(-1, 1)}


@torch.no_grad()
def soft_update(target: torch.nn.Module, online: torch.nn.Module) -> None:
    """target <- target / 2 + online / 2, parameter by parameter (bdq_model/__init__.py:137-139)."""
    for (kt, t), (ko, o) in zip(target.state_dict().items(), online.state_dict().items()):
        t.div_(2).add_(o / 2)


class _TDLoss(torch.autograd.Function):
    """pbn_bdq_td_loss: the TD loss of bdq_update on raw head outputs and its gradient in one HIP
    launch (forward computes both; backward scales the stored gradient)."""

    @staticmethod
    def forward(ctx, online, target_heads, actions, rewards, masks, gamma):
        H, rows, A = online.shape
        B = rows // 2
        loss = torch.empty(1, dtype=torch.float32, device=online.device)
        grad = torch.empty_like(online)
        scratch = torch.empty((B + 7) // 8, dtype=torch.float32, device=online.device)
        L = _lib.load()
        with torch.cuda.device(online.device):
            _lib.check(L.pbn_bdq_td_loss(online.data_ptr(), target_heads.data_ptr(), actions.data_ptr(),
                                         rewards.data_ptr(), masks.data_ptr(), B, H - 1, A, float(gamma),
                                         loss.data_ptr(), grad.data_ptr(), scratch.data_ptr(),
                                         torch.cuda.current_stream(online.device).cuda_stream), "pbn_bdq_td_loss")
        ctx.save_for_backward(grad)
        return loss[0]

    @staticmethod
    def backward(ctx, grad_out):
        (grad,) = ctx.saved_tensors
        return grad * grad_out, None, None, None, None, None


def bdq_update(q: torch.nn.Module, target: torch.nn.Module, opt: torch.optim.Optimizer, batch: Dict[str, torch.Tensor],
               gamma: float = 0.999, grad_clamp: float = 1.0, target_weights=None) -> torch.Tensor:
    """One update_policy step (bdq_model/__init__.py:111-131) on a gathered batch; returns the loss.
    On the GPU the duelings, the double-DQN target, the MSE and their backward run as one HIP
    launch on the raw head outputs (``pbn_bdq_td_loss``); elsewhere (CPU tensors) as PyTorch
    expressions.  ``target_weights``: the target network's ``head_weights()`` computed beforehand
    (it changes only at soft updates)."""
    # q(obs) and q(next_obs) as one forward over 2B rows (half the launches; only the first
    # half carries gradient)
    B = batch["obs"].shape[1]
    x = batch["x"] if "x" in batch else torch.cat([batch["obs"], batch["next_obs"]], 1)
    if x.is_cuda and isinstance(q, BranchingQNetwork) and isinstance(target, BranchingQNetwork):
        heads = q.forward_heads(q.model[0](x))                          # (K+1, 2B, A), raw
        with torch.no_grad():
            t_heads = target.forward_heads(target.model[0](batch["next_obs"]),
                                           weights=target_weights).contiguous()   # (K+1, B, A)
        loss = _TDLoss.apply(heads.contiguous(), t_heads, batch["actions"].reshape(B, -1).contiguous(),
                             batch["rewards"].reshape(B).contiguous(), batch["masks"].reshape(B).contiguous(), gamma)
    else:
        q_all = q(x)                                                    # (2B, K, A)
        current = q_all[:B].gather(2, batch["actions"]).squeeze(-1)     # (B, K)
        with torch.no_grad():
            argmax = torch.argmax(q_all[B:].detach(), dim=2)
            max_next = target(batch["next_obs"]).gather(2, argmax.unsqueeze(2)).squeeze(-1)
        expected = batch["rewards"] + max_next * gamma * batch["masks"]
        loss = F.mse_loss(expected, current)
    opt.zero_grad()
    loss.backward()
    grads = [p.grad for p in q.parameters() if p.grad is not None]
    torch._foreach_clamp_min_(grads, -grad_clamp)      # two multi-tensor launches, not one per tensor
    torch._foreach_clamp_max_(grads, grad_clamp)
    opt.step()
    return loss.detach()


def bdq_layout(n_nodes: int, n_branches: int) -> List[int]:
    """pbn_bdq_layout: the float offsets of the flat parameter buffer's 12 segments, then its size."""
    L = _lib.load()
    off = (ctypes.c_int64 * 13)()
    _lib.check(L.pbn_bdq_layout(n_nodes, n_branches, off), "pbn_bdq_layout")
    return list(off)


def fused_update_supported(n_nodes: int, n_branches: int, batch_size: int) -> bool:
    """Whether pbn_bdq_learn runs this shape (its workspace query accepts it): batch a multiple of
    16, n_nodes <= 127, n_branches 1..7, and the backward's LDS within one block."""
    L = _lib.load()
    nbytes = ctypes.c_int64()
    return L.pbn_bdq_learn_workspace(n_nodes, n_branches, batch_size, ctypes.byref(nbytes)) == 0


def _bdq_segments(q: BranchingQNetwork):
    """(parameter, segment, offset within the segment) in pbn_bdq_layout order."""
    m, A = q.model, q.ac_dim
    out = [(m[0].bilinear.weight, 0, 0), (m[0].bilinear.bias, 1, 0), (m[2].weight, 2, 0), (m[2].bias, 3, 0),
           (m[4].weight, 4, 0), (m[4].bias, 5, 0), (m[6].weight, 6, 0), (m[6].bias, 7, 0)]
    for h, hd in enumerate([q.value_head] + list(q.adv_heads)):
        out += [(hd[0].weight, 8, h * 64 * 32), (hd[0].bias, 9, h * 64), (hd[2].weight, 10, h * A * 64),
                (hd[2].bias, 11, h * A)]
    return out


class FusedBDQUpdate:
    """update_policy (bdq_model/__init__.py:100-139) as three HIP launches (``pbn_bdq_learn``,
    csrc/pbn_learn.hip) instead of ~100 PyTorch kernels: the online and target networks' forwards,
    the double-DQN TD loss, the backward, the gradient clamp and the Adam step.

    The networks' parameters move into one flat fp32 buffer each (``pbn_bdq_layout``); their
    nn.Parameters become views of it, so ``state_dict``, the PyTorch forward and the acting kernel
    see the same weights.  Each network also has an image (``q_image`` / ``t_image``, pbn_bdq_pack):
    its bilinear target table (``q_table``, the acting kernel's operand), then its dense weights
    as 16 x 16 tiles in the update kernels' MFMA-fragment orders.  The online image is rewritten by
    every update; ``pack()`` recomputes the images after weights change any other way (a loaded
    checkpoint), ``soft_update()`` moves the target network halfway (bdq_model/__init__.py:137-139)
    and repacks its image.  Adam (torch.optim.Adam's arithmetic,
    betas (0.9, 0.999), eps 1e-8) keeps its moments in buffers of the same layout and its step
    count on the device (graph-capturable)."""

    def __init__(self, q: BranchingQNetwork, target: BranchingQNetwork, net, branches: int, *, batch_size: int,
                 learning_rate: float = 1e-4, gamma: float = 0.999, grad_clamp: float = 1.0,
                 betas=(0.9, 0.999), eps: float = 1e-8, keep_grad: bool = False):
        spec = net.spec
        N = spec.n
        dev = next(q.parameters()).device
        if dev.type != "cuda":
            raise ValueError("FusedBDQUpdate runs on the GPU")
        for m in (q, target):
            if (not isinstance(m, BranchingQNetwork) or m.n != branches or m.ac_dim != N + 1
                    or m.model[0].input1_dim != N or m.model[0].input2_dim != N):
                raise ValueError("FusedBDQUpdate needs BranchingQNetwork((N, N), N + 1, branches) for both networks")
        self.net, self.N, self.K, self.B = net, N, int(branches), int(batch_size)
        self.lr, self.gamma, self.grad_clamp = float(learning_rate), float(gamma), float(grad_clamp)
        self.betas, self.eps = (float(betas[0]), float(betas[1])), float(eps)
        self.slope = float(q.model[1].negative_slope)
        self.off = bdq_layout(N, self.K)
        self.q_flat = self._flatten(q, dev)
        self.t_flat = self._flatten(target, dev)
        self.q, self.target = q, target
        self._qp, self._tp = list(q.parameters()), list(target.parameters())
        self._qv = self._tv = None
        self.m = torch.zeros_like(self.q_flat)
        self.v = torch.zeros_like(self.q_flat)
        self.step = torch.zeros(1, dtype=torch.float32, device=dev)
        n_attr = len(spec.attractors)
        L = _lib.load()
        # each network's image (pbn_bdq_pack): the bilinear target table, which the acting kernel
        # reads (q_table, a view), then the dense weights in the update kernels' fragment orders
        nimg = ctypes.c_int64()
        _lib.check(L.pbn_bdq_image_floats(net.handle, self.K, ctypes.byref(nimg)), "pbn_bdq_image_floats")
        self.q_image = torch.zeros(nimg.value, dtype=torch.float32, device=dev)
        self.t_image = torch.zeros_like(self.q_image)
        nt = n_attr * N * 256
        self.q_table = self.q_image[:nt].view(n_attr, N, 16, 16)
        self.t_table = self.t_image[:nt].view(n_attr, N, 16, 16)
        nbytes = ctypes.c_int64()
        _lib.check(L.pbn_bdq_learn_workspace(N, self.K, self.B, ctypes.byref(nbytes)), "pbn_bdq_learn_workspace")
        self.work = torch.empty((nbytes.value + 3) // 4, dtype=torch.float32, device=dev)
        self.loss = torch.zeros(1, dtype=torch.float32, device=dev)
        self.grad = torch.zeros_like(self.q_flat) if keep_grad else None
        H, A = self.K + 1, N + 1
        o = self.off
        self._acting = (None, self.q_flat[o[1]:o[1] + 256],
                        (self.q_flat[o[8]:o[8] + H * 64 * 32].view(H * 64, 32), self.q_flat[o[9]:o[9] + H * 64],
                         self.q_flat[o[10]:o[10] + H * A * 64].view(H, A, 64),
                         self.q_flat[o[11]:o[11] + H * A].view(H, 1, A)),
                        self.q_table)
        self.pack()

    def _flatten(self, q: BranchingQNetwork, dev) -> torch.Tensor:
        flat = torch.zeros(self.off[12], dtype=torch.float32, device=dev)
        with torch.no_grad():
            for p, seg, extra in _bdq_segments(q):
                at = self.off[seg] + extra
                view = flat[at:at + p.numel()].view(p.shape)
                view.copy_(p.detach())
                p.data = view
        return flat

    def _stream(self):
        return torch.cuda.current_stream(self.q_flat.device).cuda_stream

    @staticmethod
    def _versions(params) -> tuple:
        return tuple(p._version for p in params)

    @staticmethod
    def _bump(params) -> None:
        """Mark parameters the HIP kernels rewrote in place (their version counters are how
        PyTorch, and BatchedBDQ's eval-mode pack cache, see an in-place change)."""
        for p in params:
            torch.autograd.graph.increment_version(p)

    def pack(self, which: str = "both") -> None:
        """Recompute the images (pbn_bdq_pack: the bilinear target table and the fragment-ordered
        dense weights) of the online and/or target network."""
        L = _lib.load()
        with torch.cuda.device(self.q_flat.device):
            for name, flat, image in (("online", self.q_flat, self.q_image), ("target", self.t_flat, self.t_image)):
                if which in ("both", name):
                    _lib.check(L.pbn_bdq_pack(self.net.handle, self.K, flat.data_ptr(), image.data_ptr(),
                                              self._stream()), "pbn_bdq_pack")
        if which in ("both", "online"):
            self._qv = self._versions(self._qp)
        if which in ("both", "target"):
            self._tv = self._versions(self._tp)

    def sync(self) -> None:
        """Repack the table of a network whose parameters changed since its last pack (e.g. a
        load_state_dict: the copy bumps the parameters' versions); a no-op otherwise."""
        if self._versions(self._qp) != self._qv:
            self.pack("online")
        if self._versions(self._tp) != self._tv:
            self.pack("target")

    def mark_updated(self) -> None:
        """After a pbn_bdq_learn launch (eager, or a replayed graph holding one): the online
        parameters changed in place."""
        self._bump(self._qp)
        self._qv = self._versions(self._qp)

    def soft_update(self) -> None:
        """target <- target / 2 + online / 2 (soft_update's arithmetic, one pass over the buffer)."""
        with torch.no_grad():
            self.t_flat.div_(2).add_(self.q_flat / 2)
        self._bump(self._tp)
        self.pack("target")

    def acting_pack(self):
        """BatchedBDQ's weight-derived operands as views of the flat buffer (no assembly kernels)."""
        return self._acting

    def update(self, replay: "DeviceReplay", idx: torch.Tensor, advance=None) -> torch.Tensor:
        """One update on ring rows ``idx`` (int64, ``batch_size`` of them); returns the loss buffer
        (overwritten by the next update).  ``advance``: an ``_lib.FrameAdvance`` whose counters
        the update's last launch advances (and the next frame's rows it draws; BDQLearner's
        captured frame)."""
        if idx.shape != (self.B,) or idx.dtype != torch.int64:
            raise ValueError(f"idx must be {self.B} int64 ring indices")
        self.sync()
        L = _lib.load()
        b1, b2 = self.betas
        with torch.cuda.device(self.q_flat.device):
            _lib.check(L.pbn_bdq_learn(self.net.handle, self.B, idx.contiguous().data_ptr(), replay.capacity,
                                       replay.state.data_ptr(), replay.next_state.data_ptr(), replay.target.data_ptr(),
                                       replay.action.data_ptr(), self.K, replay.reward.data_ptr(),
                                       replay.done.data_ptr(), self.q_flat.data_ptr(), self.q_image.data_ptr(),
                                       self.t_flat.data_ptr(), self.t_image.data_ptr(), self.m.data_ptr(),
                                       self.v.data_ptr(), self.step.data_ptr(), self.lr, b1, b2, self.eps, self.gamma,
                                       self.grad_clamp, self.slope, self.work.data_ptr(), self.work.numel() * 4,
                                       self.loss.data_ptr(), self.grad.data_ptr() if self.grad is not None else None,
                                       ctypes.byref(advance) if advance is not None else None,
                                       self._stream()), "pbn_bdq_learn")
        if not torch.cuda.is_current_stream_capturing():
            self.mark_updated()   # (a captured update is marked by each replay: BDQLearner._replay_frame)
        return self.loss[0]

    def grads(self) -> List[torch.Tensor]:
        """The last update's clamped gradient (keep_grad=True) as views shaped like q.parameters()."""
        if self.grad is None:
            raise ValueError("construct with keep_grad=True")
        g = {id(p): self.grad[self.off[seg] + extra:self.off[seg] + extra + p.numel()].view(p.shape)
             for p, seg, extra in _bdq_segments(self.q)}
        return [g[id(p)] for p in self.q.parameters()]


class BDQLearner:
    """BranchingDQN.learn (bdq_model/__init__.py:150-238) over a VectorPBNEnv: every frame acts
    for all envs (BatchedBDQ), appends their transitions to the device replay, and, once
    ``learning_starts`` transitions are stored, takes ``updates_per_frame`` update_policy steps.
    Exploration decays linearly from ``epsilon_start`` to ``epsilon_final`` over
    ``epsilon_decay`` frames after ``learning_starts`` (decrement_epsilon, :141-148).

    ``fused`` (default: whenever the network is the reference's BranchingQNetwork on the GPU and
    the batch is a multiple of 16) runs each update as FusedBDQUpdate's three HIP launches; the
    Adam state is then FusedBDQUpdate's and ``opt`` is None.  ``fused=False`` keeps the PyTorch
    update (bdq_update + torch.optim.Adam)."""

    def __init__(self, env: VectorPBNEnv, qnet: Optional[BranchingQNetwork] = None, *, capacity: int = 10 ** 4,
                 batch_size: int = 256, learning_rate: float = 1e-4, gamma: float = 0.999,
                 target_update: int = 10_000, learning_starts: int = 288, updates_per_frame: int = 1,
                 epsilon_start: float = 1.0, epsilon_final: float = 0.0, epsilon_decay: int = 10_000, seed: int = 0,
                 graphable: bool = False, blas: Optional[str] = "cublas", fused: Optional[bool] = None):
        if not env.keep_final_state:
            raise ValueError("BDQLearner needs the env's final_state (keep_final_state=True)")
        self.env = env
        self.agent = BatchedBDQ(env, qnet)
        self.q = self.agent.q.train()
        self.target = BranchingQNetwork((env.n_nodes, env.n_nodes), env.n_nodes + 1, self.agent.branches).to(env.device)
        self.target.load_state_dict(self.q.state_dict())
        can_fuse = (env.device.type == "cuda" and self.agent.fused_tail and isinstance(self.q, BranchingQNetwork)
                    and fused_update_supported(env.n_nodes, self.agent.branches, batch_size))
        if fused and not can_fuse:
            raise ValueError("fused update: the reference BranchingQNetwork on a GPU env, batch a multiple of 16")
        self.fused: Optional[FusedBDQUpdate] = None
        self.opt = None
        if fused if fused is not None else can_fuse:
            self.fused = FusedBDQUpdate(self.q, self.target, env.net, self.agent.branches, batch_size=batch_size,
                                        learning_rate=learning_rate, gamma=gamma)
            self.agent.pack_provider = self.fused.acting_pack
        else:
            if blas:
                # the PyTorch update's GEMMs are small (batch 256-512, widths 28-256): rocBLAS
                # ("cublas" in torch's naming on ROCm) runs the weight-gradient products (K = batch)
                # 2.5-8x faster than hipBLASLt's picks (tools/learn_profile.py, profiles/r04_z*).
                # This sets the process-wide preference, so only this path sets it (the fused
                # update runs no GEMM); blas=None leaves it alone
                torch.backends.cuda.preferred_blas_library(blas)
            # one fused multi-tensor kernel per step instead of a handful per parameter tensor
            # capturable keeps Adam's step counts on the device (needed to replay it in a hipGraph)
            self.opt = torch.optim.Adam(self.q.parameters(), lr=learning_rate, fused=True, capturable=graphable)
        self.replay = DeviceReplay(max(capacity, env.n_alloc), env.words, self.agent.branches, env.device)
        self.batch_size, self.gamma, self.target_update = batch_size, gamma, target_update
        self.learning_starts = max(learning_starts, batch_size)
        self.updates_per_frame = updates_per_frame
        self.epsilon = epsilon_start
        self.epsilon_final = epsilon_final
        self.epsilon_step = (epsilon_start - epsilon_final) / max(1, epsilon_decay)
        self.frames = 0
        self.updates = 0
        self.gen = torch.Generator(device=env.device)
        self.gen.manual_seed(seed)
        self.seed = int(seed)
        if self.fused is not None:
            # the fused learner draws its rows from the REPLAY Philox stream (pbn_replay_advance):
            # all updates_per_frame batches of a frame in one draw, eager or captured
            self._draw_t = torch.zeros(1, dtype=torch.int64, device=env.device)
            self._idx = torch.empty(updates_per_frame * batch_size, dtype=torch.int64, device=env.device)
        self.last_loss: Optional[torch.Tensor] = None
        self.graphable = graphable
        self._graph: Optional[torch.cuda.CUDAGraph] = None
        self._tw = None   # _target_weights()
        self._tw_key = None

    def _target_weights(self):
        """The target network's stacked head weights (BranchingQNetwork.head_weights), held in
        fixed tensors (a captured frame reads these very tensors).  They are refreshed in place
        whenever the target's parameters changed since (soft updates, a load_state_dict: any
        in-place write bumps the parameters' versions)."""
        key = tuple(p._version for p in self.target.parameters())
        if self._tw is None:
            with torch.no_grad():
                self._tw = tuple(w.detach().clone() for w in self.target.head_weights())
        elif key != self._tw_key:
            self._refresh_target_weights()
        self._tw_key = key
        return self._tw

    def _refresh_target_weights(self) -> None:
        if self._tw is not None:
            with torch.no_grad():
                for dst, w in zip(self._tw, self.target.head_weights()):
                    dst.copy_(w)
            self._tw_key = tuple(p._version for p in self.target.parameters())

    def frame(self):
        if self._graph is not None:
            return self._replay_frame()
        env = self.env
        state = env.state.clone()
        target = env.target.clone()
        self.agent.act_q(self.epsilon)
        _, reward, flags = env.step_flipmask(use_current=True)
        done_all = (env.flags & (_lib.FLAG_TERMINATED | _lib.FLAG_TRUNCATED)) != 0
        # all n_alloc envs are stored (the padding envs of a ragged batch are real envs too)
        self.replay.store(state, target, self.agent.actions, env.reward, env.final_state, done_all)
        done = done_all[: env.num_envs]
        self.frames += 1
        if self.replay.size >= self.learning_starts:
            self.epsilon = max(self.epsilon_final, self.epsilon - self.epsilon_step)
            if self.fused is not None:
                size_t = torch.full((1,), self.replay.size, dtype=torch.int64, device=env.device)
                self.replay.sample_rows(self._idx, self.seed, self._draw_t, size_t)
            for u in range(self.updates_per_frame):
                if self.fused is not None:
                    self.last_loss = self.fused.update(self.replay, self._idx[u * self.batch_size:(u + 1) * self.batch_size])
                else:
                    self.last_loss = self._update(self.replay.sample_indices(self.batch_size, self.gen))
                self.updates += 1
                if self.updates % self.target_update == 0:
                    self._soft_update()
        return reward, done

    def refresh_weights(self) -> None:
        """Call after changing ``q`` / ``target`` weights outside frame() (e.g. loading a reference
        checkpoint, bdq_model/__init__.py:244, with load_state_dict): repacks the fused update's
        bilinear target tables, or the PyTorch path's cached target head weights.  A captured
        frame reads the same buffers, so it needs no re-capture."""
        if self.fused is not None:
            self.fused.pack()
        else:
            self._refresh_target_weights()

    def _update(self, idx: torch.Tensor) -> torch.Tensor:
        if self.fused is not None:
            return self.fused.update(self.replay, idx)
        batch = self.replay.gather(idx, self.env.net)
        return bdq_update(self.q, self.target, self.opt, batch, self.gamma, target_weights=self._target_weights())

    def _soft_update(self) -> None:
        if self.fused is not None:
            self.fused.soft_update()
        else:
            soft_update(self.target, self.q)
            self._refresh_target_weights()

    # ---- graph-captured frames -------------------------------------------------------------
    def capture(self, min_updates: int = 3) -> None:
        """Capture one whole learning frame (obs unpack, Q forward, epsilon-greedy flip masks,
        pbn_step_dev, replay store, epsilon decay, ``updates_per_frame`` update_policy steps)
        in a hipGraph; ``frame()`` replays it from then on.  The step index, epsilon, ring
        position and fill level live in device tensors the graph advances, mirrored on the
        host after every replay; target-network soft updates stay on the host (between
        replays), so ``target_update`` must be a multiple of ``updates_per_frame``.

        Frames run eagerly (on a side stream, as graph capture requires) until learning has
        started and ``min_updates`` updates have initialised Adam's state and library
        workspaces.  After capture, the env must only be stepped through ``frame()``."""
        if not self.graphable:
            raise ValueError("construct the learner with graphable=True to capture it")
        if self.target_update % self.updates_per_frame:
            raise ValueError("target_update must be a multiple of updates_per_frame")
        env = self.env
        dev = env.device
        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            while self.replay.size < self.learning_starts or self.updates < min_updates:
                self.frame()
        torch.cuda.current_stream(dev).wait_stream(side)
        self._step_t = torch.full((1,), env.step_index, dtype=torch.int64, device=dev)
        self._eps64 = torch.full((1,), self.epsilon, dtype=torch.float64, device=dev)
        self._eps32 = self._eps64.float()
        self._pos_t = torch.full((1,), self.replay.pos, dtype=torch.int64, device=dev)
        self._size_t = torch.full((1,), self.replay.size, dtype=torch.int64, device=dev)
        self._done_buf = torch.zeros(env.n_alloc, dtype=torch.uint8, device=dev)
        self._tgt_prev = env.target.clone()   # the pre-step targets, carried by the ring store
        # under the one-update law the step kernel writes the ring rows itself (pbn_step_dev_store)
        self._ring = None
        if env.spec.settle < 2:
            rp = self.replay
            self._ring = _lib.RingStore(
                rp.capacity, self._pos_t.data_ptr(), rp.state.data_ptr(), rp.next_state.data_ptr(), rp.target.data_ptr(),
                rp.action.data_ptr(), rp.reward.data_ptr(), rp.done.data_ptr(), self.agent.actions.data_ptr(),
                rp.action.shape[1], _lib.FLAG_TERMINATED | _lib.FLAG_TRUNCATED, self._done_buf.data_ptr())
        self._adv = None
        if self.fused is not None:
            # the fused update's last launch advances the frame's counters and draws the next
            # frame's rows (pbn_frame_advance): the first replayed frame's rows are drawn now, over
            # the fill level its store will leave (what pbn_replay_advance drew inside the frame)
            self._adv = _lib.FrameAdvance(
                env.n_alloc, self.replay.capacity, self._pos_t.data_ptr(), self._size_t.data_ptr(),
                self._step_t.data_ptr(), self._eps64.data_ptr(), self._eps32.data_ptr(), float(self.epsilon_final),
                float(self.epsilon_step), self._idx.numel(), self.seed, self._draw_t.data_ptr(), self._idx.data_ptr())
            first = torch.full((1,), min(self.replay.size + env.n_alloc, self.replay.capacity), dtype=torch.int64,
                               device=dev)
            self.replay.sample_rows(self._idx, self.seed, self._draw_t, first)
        g = torch.cuda.CUDAGraph()
        g.register_generator_state(self.gen)
        if self.opt is not None:
            self.opt.zero_grad(set_to_none=True)
        with torch.cuda.graph(g):
            self._g_out = self._graph_body()
        self._graph = g
        # the capture recorded the frame without running it: nothing above advanced
        torch.cuda.current_stream(dev).synchronize()

    def _graph_body(self):
        env = self.env
        self.agent.act_q(step_t=self._step_t, epsilon_t=self._eps32)
        if self._ring is not None:
            # one launch: the step, in place, writing its transitions into the ring
            env.step_flipmask_dev_store(self._step_t, self._ring)
        else:
            env.step_flipmask_dev(self._step_t, copy_back=False)
            # the ring store reads the pre-step state (still in env.state) and target (carried in
            # _tgt_prev), derives done from the flags, and in the same pass moves the stepped state
            # into env.state and the new targets into _tgt_prev
            self.replay.store_at(self._pos_t, self._size_t, env.state, self._tgt_prev, self.agent.actions,
                                 env.reward, env.final_state, env.flags,
                                 done_mask=_lib.FLAG_TERMINATED | _lib.FLAG_TRUNCATED, done_out=self._done_buf,
                                 advance=False, state_copy=(env.state, env._state_next),
                                 target_copy=(self._tgt_prev, env.target))
        # then the counters: the step index, the ring position and fill level, epsilon (and, fused,
        # the next frame's rows) advance in the update's last launch or in pbn_replay_advance
        fused = self.fused is not None
        L = _lib.load()
        if not fused:   # (fused: the update's last launch advances them, pbn_frame_advance)
            with torch.cuda.device(env.device):
                _lib.check(L.pbn_replay_advance(env.n_alloc, self.replay.capacity, self._pos_t.data_ptr(),
                                                self._size_t.data_ptr(), self._step_t.data_ptr(),
                                                self._eps64.data_ptr(), self._eps32.data_ptr(),
                                                float(self.epsilon_final), float(self.epsilon_step), 0, self.seed,
                                                None, None, torch.cuda.current_stream(env.device).cuda_stream),
                           "pbn_replay_advance")
        loss = None
        B = self.batch_size
        U = self.updates_per_frame
        for u in range(U):
            if fused:
                loss = self.fused.update(self.replay, self._idx[u * B:(u + 1) * B],
                                         advance=self._adv if u == U - 1 else None)
            else:
                loss = self._update(self.replay.sample_indices(B, self.gen, size_t=self._size_t))
        return env.reward[: env.num_envs], self._done_buf[: env.num_envs].view(torch.bool), loss

    def _replay_frame(self):
        env, rp = self.env, self.replay
        if self.fused is not None:
            self.fused.sync()            # weights loaded between replays: repack the tables
        else:
            self._target_weights()       # (refreshes the captured head-weight copies if stale)
        self._graph.replay()
        # the replayed update rewrote the online parameters in place (version counters: what
        # PyTorch and BatchedBDQ's eval-mode pack cache read)
        if self.fused is not None:
            self.fused.mark_updated()
        else:
            FusedBDQUpdate._bump(self.q.parameters())
        env.step_index += 1
        rp.pos = (rp.pos + env.n_alloc) % rp.capacity
        rp.size = min(rp.size + env.n_alloc, rp.capacity)
        self.epsilon = max(self.epsilon_final, self.epsilon - self.epsilon_step)
        self.frames += 1
        self.updates += self.updates_per_frame
        if self.updates % self.target_update == 0:
            self._soft_update()
        reward, done, self.last_loss = self._g_out
        return reward, done

