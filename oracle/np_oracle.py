"""numpy restatement of the batched step, vectorised over envs (one process, one core).

TEST INFRASTRUCTURE ONLY: imported by tests/ (checked against oracle/pbn_oracle.c) and by
bench.py's CPU-baseline leg, as the batched numpy restatement SURVEY.md 8(d)(ii) asks for.
It restates DESIGN.md "Step semantics" the way oracle/pyoracle.py does (that file's
PyPBN.step is the per-env form: same draws, same order), but for all envs at once:
loops run over nodes, digit planes and gap draws, never over envs.  The reference's own
step is gym_PBN's external per-node loop behind env.step (bdq_model/__init__.py:177);
the semantics it freezes are SURVEY.md Appendix C.
"""
from __future__ import annotations

import numpy as np

from oracle.agent_oracle import philox_vec

SEL, ENV, PERT, RESET = 0, 1, 2, 3
MODE_AUTORESET, MODE_RANDOM_ACTIONS = 1, 2
_U32 = np.uint64(0xFFFFFFFF)


def _draw(seed: int, ident: np.ndarray, step: int, stream: int, idx) -> list:
    """Philox words (4 arrays) keyed (ident, step, stream << 28 | idx) -- pyoracle.draw, batched."""
    ident = np.asarray(ident, dtype=np.uint64)
    c0 = ident & _U32
    c1 = np.full(ident.shape, step & 0xFFFFFFFF, dtype=np.uint64)
    c2 = (np.uint64(stream << 28) | (np.asarray(idx, dtype=np.uint64) & np.uint64(0x0FFFFFFF))) + np.zeros_like(ident)
    c3 = ((ident >> np.uint64(32)) & np.uint64(0xFFFF)) | np.uint64(((step >> 32) & 0xFFFF) << 16)
    return philox_vec(c0, c1, c2, c3, seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF)


def ext64(hi: np.ndarray, lo: np.ndarray, k):
    """Bounded draws from 64-bit uniforms (hi:lo) (pyoracle.ext64, batched): returns
    (floor(x * k / 2^64), hi', lo') with x' = x * k mod 2^64; k < 2^32 scalar or per env."""
    k = np.asarray(k, dtype=np.uint64)
    a = lo.astype(np.uint64) * k                          # < 2^64
    b = hi.astype(np.uint64) * k + (a >> np.uint64(32))   # < 2^64
    return (b >> np.uint64(32)).astype(np.int64), (b & _U32).astype(np.uint32), (a & _U32).astype(np.uint32)


class NpPBN:
    """Batched env semantics over an EnvSpec (network + attractors + constants)."""

    def __init__(self, spec):
        self.spec = spec
        self.net = spec.network
        self.n = self.net.n
        self.W = spec.words
        self.thr = [np.asarray(t, dtype=np.int64) for t in self.net.thresholds(spec.prob_bits)]
        self.cdf = np.asarray(spec.arrays["perturb_cdf"], dtype=np.uint64)
        # functions as (inputs, truth-table bit array) for vectorised lookup
        self.funcs = []
        for fl in self.net.nodes:
            row = []
            for f in fl:
                k = len(f.inputs)
                nbytes = max(1, (1 << k) // 8)
                bits = np.unpackbits(np.frombuffer(int(f.table).to_bytes(nbytes, "little"), dtype=np.uint8),
                                     bitorder="little")[: 1 << k].astype(np.uint32)
                row.append((list(f.inputs), bits))
            self.funcs.append(row)
        # attractor states packed to words, sorted by a 64-bit mixing hash for searchsorted
        self.att_words, self.att_id, self.att_first, self.att_len = [], [], [], []
        for a, att in enumerate(spec.attractors):
            self.att_first.append(len(self.att_words))
            self.att_len.append(len(att))
            for s in att:
                self.att_words.append(self._pack_bits(s))
                self.att_id.append(a)
        self.att_words = np.asarray(self.att_words, dtype=np.uint32).reshape(-1, self.W)
        self.att_id = np.asarray(self.att_id, dtype=np.int64)
        h = self._hash(self.att_words.T)
        self.order = np.argsort(h, kind="stable")
        self.hsorted = h[self.order]
        A = len(spec.attractors)
        self.A = A
        pcs = np.arange(self.n + 1)
        self.rtab = np.asarray([[spec.reward_value(term, wrong, int(p)) for p in pcs]
                                for term, wrong in ((False, False), (False, True), (True, False))],
                               dtype=np.float32)

    def _pack_bits(self, bits):
        words = [0] * self.W
        for i, v in enumerate(bits):
            if int(v):
                words[i >> 5] |= 1 << (i & 31)
        return words

    @staticmethod
    def _hash(words: np.ndarray) -> np.ndarray:
        """words (W, n) uint32 -> uint64 mixing hash per env."""
        h = np.zeros(words.shape[1], dtype=np.uint64)
        with np.errstate(over="ignore"):
            for w in range(words.shape[0]):
                h = (h ^ words[w].astype(np.uint64)) * np.uint64(0x9E3779B97F4A7C15)
                h ^= h >> np.uint64(29)
        return h

    def attractor_of(self, words: np.ndarray) -> np.ndarray:
        """(W, n) packed states -> attractor id per env, or -1."""
        n = words.shape[1]
        out = np.full(n, -1, dtype=np.int64)
        if len(self.att_id) == 0:
            return out
        h = self._hash(words)
        pos = np.searchsorted(self.hsorted, h, side="left")
        # walk the (rare) runs of equal hashes until the words match
        while True:
            live = (out < 0) & (pos < len(self.hsorted))
            live[live] &= self.hsorted[pos[live]] == h[live]
            if not live.any():
                break
            cand = self.order[pos[live]]
            eq = np.all(self.att_words[cand].T == words[:, live], axis=0)
            idx = np.nonzero(live)[0]
            out[idx[eq]] = self.att_id[cand[eq]]
            pos[idx[~eq]] += 1
            pos[idx[eq]] = len(self.hsorted)
        return out

    def _bit(self, words: np.ndarray, i: int) -> np.ndarray:
        return (words[i >> 5] >> np.uint32(i & 31)) & np.uint32(1)

    def reset_draw(self, hi: np.ndarray, lo: np.ndarray):
        """Attractor draws from the 64-bit uniforms (hi:lo) per env (pyoracle.reset_draw; A >= 1):
        (state words (W, n), target ids (n,), hi', lo')."""
        n = len(hi)
        A = self.A
        a_s = np.zeros(n, dtype=np.int64)
        a_t = np.zeros(n, dtype=np.int64)
        if A >= 2:
            c, hi, lo = ext64(hi, lo, A * (A - 1))
            a_s, a_t = c // (A - 1), c % (A - 1)
            a_t += (a_t >= a_s)
        size = np.asarray(self.att_len, dtype=np.int64)[a_s]
        idx, hi, lo = ext64(hi, lo, size)
        rows = np.asarray(self.att_first, dtype=np.int64)[a_s] + idx
        state = self.att_words[rows].T.copy()
        return state, a_t.astype(np.uint8), hi, lo

    def random_state(self, seed: int, e: np.ndarray, step: int):
        n = len(e)
        r = _draw(seed, e, step, RESET, 1)
        state = np.zeros((self.W, n), dtype=np.uint32)
        for w in range(self.W):
            nb = min(32, self.n - 32 * w)
            state[w] = r[w] & np.uint32(0xFFFFFFFF if nb == 32 else (1 << nb) - 1)
        return state, np.full(n, 0xFF, dtype=np.uint8)

    def reset_from_words(self, seed: int, e: np.ndarray, step: int, hi: np.ndarray, lo: np.ndarray):
        """pbn_reset's draw: (state words (W, n), target ids (n,)) from the 64-bit uniform (hi:lo)
        per env (pyoracle.reset_from_words)."""
        if self.A >= 1:
            state, tgt, _, _ = self.reset_draw(hi, lo)
            return state, tgt
        return self.random_state(seed, e, step)

    def reset(self, seed: int, step: int, env_offset: int, n: int):
        e = np.arange(n, dtype=np.uint64) + np.uint64(env_offset)
        R = _draw(seed, e, step, RESET, 0)
        state, tgt = self.reset_from_words(seed, e, step, R[1], R[0])
        return state, tgt, np.zeros(n, dtype=np.uint8)

    def step(self, seed: int, step: int, env_offset: int, state, flipmask, target, t, mode: int) -> dict:
        n_nodes, B, W = self.n, self.spec.prob_bits, self.W
        state = np.asarray(state, dtype=np.uint32)
        n = state.shape[1]
        e = np.arange(n, dtype=np.uint64) + np.uint64(env_offset)
        # one ENV call: words 0, 1 = gaps 0, 1; X = words 3:2 gives, in order, the action draw
        # (every mode), the autoreset draws and gap 2's uniform (pyoracle.step)
        E = _draw(seed, e, step, ENV, 0)
        c, hi, lo = ext64(E[3], E[2], (n_nodes + 1) ** 3)
        reset_to = None
        if self.A >= 1:
            rs, rt, hi, lo = self.reset_draw(hi, lo)
            reset_to = (rs, rt)
        u2 = hi
        if mode & MODE_RANDOM_ACTIONS:
            flip = np.zeros((W, n), dtype=np.uint32)
            for k in range(3):
                c, a = c // (n_nodes + 1), c % (n_nodes + 1)
                for w in range(W):
                    sel = (a > 0) & (((a - 1) >> 5) == w)
                    flip[w, sel] |= (np.uint32(1) << ((a[sel] - 1) & 31).astype(np.uint32))
        else:
            flip = np.asarray(flipmask, dtype=np.uint32).copy()
        s1 = state ^ flip
        # perturbation: geometric gaps from ENV words 0, 1, u2, then PERT calls
        gamma = np.zeros((W, n), dtype=np.uint32)
        pos = np.full(n, -1, dtype=np.int64)
        live = np.ones(n, dtype=bool)
        k, P = 0, None
        while live.any():
            if k < 2:
                u = E[k]
            elif k == 2:
                u = u2
            else:
                if (k - 3) % 4 == 0:
                    P = _draw(seed, e, step, PERT, (k - 3) // 4)
                u = P[(k - 3) % 4]
            k += 1
            gap = np.searchsorted(self.cdf, u.astype(np.uint64), side="right") + 1
            pos = np.where(live, pos + gap, pos)
            hit = live & (pos < n_nodes)
            for w in range(W):
                m = hit & ((pos >> 5) == w)
                gamma[w, m] |= np.uint32(1) << (pos[m] & 31).astype(np.uint32)
            live = hit & (pos < n_nodes - 1)
        perturbed = np.any(gamma != 0, axis=0)
        # node updates from s1: selection u per (group, node) from SEL digit planes
        G = e >> np.uint64(5)
        b = (e & np.uint64(31)).astype(np.uint32)
        ug, ginv = np.unique(G, return_inverse=True)
        sp = np.zeros((W, n), dtype=np.uint32)
        for i, fl in enumerate(self.funcs):
            if len(fl) == 1:
                j = np.zeros(n, dtype=np.int64)
            else:
                u = np.zeros(n, dtype=np.int64)
                for c in range((B + 3) // 4):
                    words = _draw(seed, ug, step, SEL, 4 * i + c)
                    for q in range(4):
                        d = 4 * c + q
                        if d >= B:
                            break
                        bit = (words[q][ginv] >> b) & np.uint32(1)
                        u |= bit.astype(np.int64) << (B - 1 - d)
                thr = self.thr[i]
                j = np.zeros(n, dtype=np.int64)
                for jj in range(len(fl) - 1):   # first j with u < thr[j], else the last function
                    j += (j == jj) & ~(u < thr[jj])
            x = np.zeros(n, dtype=np.uint32)
            for jj, (ins, bits) in enumerate(fl):
                m = j == jj
                if not m.any():
                    continue
                idx = np.zeros(int(m.sum()), dtype=np.int64)
                for q, g in enumerate(ins):
                    idx |= self._bit(s1[:, m], g).astype(np.int64) << q
                x[m] = bits[idx]
            sp[i >> 5] |= x << np.uint32(i & 31)
        sp = np.where(perturbed[None, :], s1 ^ gamma, sp).astype(np.uint32)
        att = self.attractor_of(sp)
        in_attr = att >= 0
        tgt = np.asarray(target, dtype=np.uint8).copy()
        term = in_attr & (att == tgt.astype(np.int64))
        tt = np.minimum(np.asarray(t, dtype=np.int64) + 1, 255)
        hz = self.spec.horizon
        trunc = (tt >= hz) if hz > 0 else np.zeros(n, dtype=bool)
        wrong = in_attr & ~term
        pc = np.zeros(n, dtype=np.int64)
        for w in range(W):
            pc += np.unpackbits(flip[w].view(np.uint8).reshape(n, 4), axis=1).sum(axis=1, dtype=np.int64)
        case = np.where(term, 2, np.where(wrong, 1, 0))
        reward = self.rtab[case, pc]
        flags = (term.astype(np.uint8) | (trunc.astype(np.uint8) << 1) | (in_attr.astype(np.uint8) << 2)
                 | (perturbed.astype(np.uint8) << 3))
        state_out = sp.copy()
        t_out = tt.astype(np.uint8)
        if mode & MODE_AUTORESET:
            done = term | trunc
            if done.any():
                if reset_to is not None:
                    ns, ntg = reset_to[0][:, done], reset_to[1][done]
                else:
                    ns, ntg = self.random_state(seed, e[done], step)
                state_out[:, done] = ns
                tgt[done] = ntg
                t_out[done] = 0
                flags[done] |= 16
        return {"state_out": state_out, "final_state": sp, "reward": reward, "flags": flags,
                "target": tgt, "t": t_out, "flipmask": flip}
