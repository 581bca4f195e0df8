"""Test helper: an oracle-backed stand-in for VectorPBNEnv on CPU tensors (used to
exercise the multi-rank sharding / gather logic with gloo, without a GPU)."""
import numpy as np
import torch

from oracle import oracle


class OracleVectorEnv:
    def __init__(self, spec, env_offset, count, seed=0):
        self.spec, self.env_offset, self.count, self.seed = spec, env_offset, count, seed
        self.words = spec.words
        st, tg, t = oracle.reset(spec, seed, 0, env_offset, count)
        self._st, self._tg, self._t = st, tg, t
        self.step_index = 1
        self.state = torch.from_numpy(st.view(np.int32).copy())
        self.flipmask = torch.zeros_like(self.state)
        self.final_state = torch.zeros_like(self.state)
        self.device = torch.device("cpu")

    def step_flipmask(self, flipmask=None, random_actions=False):
        flip = np.zeros_like(self._st) if flipmask is None else flipmask.numpy().view(np.uint32)
        mode = 1 | (2 if random_actions else 0)
        out = oracle.step(self.spec, self.seed, self.step_index, self.env_offset, self._st, flip, self._tg,
                          self._t, mode)
        self.step_index += 1
        self._st, self._tg, self._t = out["state_out"], out["target"], out["t"]
        self.state = torch.from_numpy(out["state_out"].view(np.int32).copy())
        self.flipmask = torch.from_numpy(out["flipmask"].view(np.int32).copy())
        self.final_state = torch.from_numpy(out["final_state"].view(np.int32).copy())
        self.updates = torch.from_numpy(out["updates"].view(np.int16).copy())
        return self.state, torch.from_numpy(out["reward"]), torch.from_numpy(out["flags"])

    def rollout(self, n_steps, flipmasks=None, random_actions=True, keep_obs=True, keep_final=True, out=None):
        """Same contract as VectorPBNEnv.rollout (dict of [n_steps, ...] tensors)."""
        W, n = self.words, self.count
        rec = out if out is not None else {
            "obs": torch.empty((n_steps, W, n), dtype=torch.int32),
            "flipmask": torch.empty((n_steps, W, n), dtype=torch.int32),
            "final_state": torch.empty((n_steps, W, n), dtype=torch.int32),
            "reward": torch.empty((n_steps, n), dtype=torch.float32),
            "flags": torch.empty((n_steps, n), dtype=torch.uint8),
            "updates": torch.empty((n_steps, n), dtype=torch.int16)}
        for k in range(n_steps):
            rec["obs"][k] = self.state
            fm = None if flipmasks is None else flipmasks[k]
            _, reward, flags = self.step_flipmask(fm, random_actions=random_actions and fm is None)
            rec["flipmask"][k] = self.flipmask
            rec["final_state"][k] = self.final_state
            rec["reward"][k] = reward
            rec["flags"][k] = flags
            if "updates" in rec:
                rec["updates"][k] = self.updates
        return rec
