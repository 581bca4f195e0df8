"""Pure-Python, one-env-at-a-time restatement of the step (gym-PBN style).

TEST INFRASTRUCTURE ONLY.  Second, independent restatement of DESIGN.md
"Step semantics": it works from the compiled ``Network`` objects (per-node
function lists, boolean tables) rather than from the C descriptor, so agreement
with oracle/pbn_oracle.c also checks the descriptor encoding.  It is slow by
construction (per-node Python loop, like the external gym_PBN step the
reference calls at bdq_model/__init__.py:177) and doubles as the
"reference-style Python" CPU baseline in bench.py.
"""
from __future__ import annotations

from typing import Dict, List, Sequence, Tuple

M0, M1 = 0xD2511F53, 0xCD9E8D57
W0, W1 = 0x9E3779B9, 0xBB67AE85
MASK32 = 0xFFFFFFFF
SEL, ENV, PERT, RESET, SETTLE_SEL, SETTLE_ENV = 0, 1, 2, 3, 5, 6
MODE_AUTORESET, MODE_RANDOM_ACTIONS = 1, 2


# every stream draws Philox4x32-7 (DESIGN.md "RNG"); the round function is pinned at 7 and 10
# rounds by known-answer vectors (tests/test_philox.py)
PHILOX_ROUNDS = 7


def philox4x32(ctr: Sequence[int], key: Sequence[int], rounds: int = PHILOX_ROUNDS) -> Tuple[int, int, int, int]:
    c0, c1, c2, c3 = (int(x) & MASK32 for x in ctr)
    k0, k1 = int(key[0]) & MASK32, int(key[1]) & MASK32
    for _ in range(rounds):
        p0 = M0 * c0
        p1 = M1 * c2
        c0, c1, c2, c3 = ((p1 >> 32) ^ c1 ^ k0) & MASK32, p1 & MASK32, ((p0 >> 32) ^ c3 ^ k1) & MASK32, p0 & MASK32
        k0 = (k0 + W0) & MASK32
        k1 = (k1 + W1) & MASK32
    return c0, c1, c2, c3


def philox4x32_10(ctr: Sequence[int], key: Sequence[int]) -> Tuple[int, int, int, int]:
    return philox4x32(ctr, key, 10)


def draw(seed: int, ident: int, step: int, stream: int, idx: int):
    ctr = (ident & MASK32, step & MASK32, (stream << 28) | (idx & 0x0FFFFFFF),
           ((ident >> 32) & 0xFFFF) | (((step >> 32) & 0xFFFF) << 16))
    return philox4x32(ctr, (seed & MASK32, (seed >> 32) & MASK32))


def ext64(x: int, k: int) -> Tuple[int, int]:
    """One bounded draw from the 64-bit uniform x: (floor(x * k / 2^64), x * k mod 2^64)."""
    prod = x * k
    return prod >> 64, prod & ((1 << 64) - 1)


class PyPBN:
    """Scalar env semantics over an EnvSpec (network + attractors + constants)."""

    def __init__(self, spec):
        self.spec = spec
        self.net = spec.network
        self.n = self.net.n
        self.thr = self.net.thresholds(spec.prob_bits)
        self.cdf = [int(x) for x in spec.arrays["perturb_cdf"]]
        self.att_of: Dict[Tuple[int, ...], int] = {}
        for a, att in enumerate(spec.attractors):
            for s in att:
                self.att_of[tuple(s)] = a

    def gap(self, u: int) -> int:
        for m in range(1, self.n + 1):
            if u < self.cdf[m - 1]:
                return m
        return self.n + 1

    def reset_draw(self, x: int):
        """Attractor draws from the 64-bit uniform x: one draw over the A(A-1) ordered (start,
        target) pairs (A >= 2), then the state uniformly within the start attractor.  Returns
        (start state, target id, what remains of x); A >= 1."""
        A = len(self.spec.attractors)
        a_s = a_t = 0
        if A >= 2:
            c, x = ext64(x, A * (A - 1))
            a_s, a_t = divmod(c, A - 1)
            a_t += a_t >= a_s
        att = self.spec.attractors[a_s]
        idx, x = ext64(x, len(att))
        return list(att[idx]), a_t, x

    def random_state(self, seed: int, e: int, step: int):
        r = draw(seed, e, step, RESET, 1)
        return [(r[i >> 5] >> (i & 31)) & 1 for i in range(self.n)], 0xFF

    def reset_from_words(self, seed: int, e: int, step: int, hi: int, lo: int):
        """pbn_reset's draw: (start state, target id) from the 64-bit uniform (hi:lo)."""
        if self.spec.attractors:
            state, tgt, _ = self.reset_draw((hi << 32) | lo)
            return state, tgt
        return self.random_state(seed, e, step)

    def reset(self, seed: int, step: int, e: int):
        R = draw(seed, e, step, RESET, 0)
        state, tgt = self.reset_from_words(seed, e, step, R[1], R[0])
        return state, tgt, 0

    def group_uniform(self, seed: int, G: int, b: int, step: int, i: int) -> int:
        """One-update law: node i's B-bit uniform for env bit b of group G, from the group's
        digit planes (SEL call 4i + c, word d & 3 = digit 4c + d, digit 0 the MSB)."""
        B, u = self.spec.prob_bits, 0
        for d in range(B):
            word = draw(seed, G, step, SEL, 4 * i + (d >> 2))[d & 3]
            u |= ((word >> b) & 1) << (B - 1 - d)
        return u

    def env_uniform(self, seed: int, e: int, step: int, k: int, i: int) -> int:
        """Settle law: node i's B-bit uniform for update k of env e's step, keyed per env: the
        top B bits of 16-bit field i & 1 of word (i >> 1) & 3 of SETTLE_SEL call (k << 8 | i >> 3)."""
        word = draw(seed, e, step, SETTLE_SEL, (k << 8) | (i >> 3))[(i >> 1) & 3]
        return ((word >> (16 * (i & 1))) & 0xFFFF) >> (16 - self.spec.prob_bits)

    def rule_update(self, s1: List[int], uniform) -> List[int]:
        """Every node's rule update from s1; uniform(i) = node i's B-bit selection uniform."""
        sp = []
        for i, fl in enumerate(self.net.nodes):
            j = 0
            if len(fl) > 1:
                u = uniform(i)
                while j < len(fl) - 1 and not (u < self.thr[i][j]):
                    j += 1
            sp.append(fl[j](s1))
        return sp

    def step(self, seed: int, step: int, e: int, state: List[int], flip: List[int], target: int, t: int,
             mode: int):
        n, B = self.n, self.spec.prob_bits
        G, b = e >> 5, e & 31
        # one ENV call: words 0, 1 = gaps 0, 1; X = words 3:2 gives, in order, the action draw
        # (every mode), the autoreset draws and gap 2's uniform (the top word of what remains)
        E = draw(seed, e, step, ENV, 0)
        c, x = ext64((E[3] << 32) | E[2], (n + 1) ** 3)   # 3 uniform ints in [0, N] (:76)
        reset_to = None
        if self.spec.attractors:
            rs, rt, x = self.reset_draw(x)
            reset_to = (rs, rt)
        u2 = x >> 32
        if mode & MODE_RANDOM_ACTIONS:
            flip = [0] * n
            for k in range(3):
                c, a = divmod(c, n + 1)
                if a > 0:
                    flip[a - 1] = 1  # each distinct node once (bdq_model/__init__.py:81-84,176)
        s1 = [state[i] ^ flip[i] for i in range(n)]
        gamma = [0] * n
        pos, k, P = -1, 0, None
        while pos < n - 1:
            if k < 2:
                u = E[k]
            elif k == 2:
                u = u2
            else:
                if (k - 3) % 4 == 0:
                    P = draw(seed, e, step, PERT, (k - 3) // 4)
                u = P[(k - 3) % 4]
            k += 1
            pos += self.gap(u)
            if pos >= n:
                break
            gamma[pos] = 1
        perturbed = any(gamma)
        settle_law = self.spec.settle >= 2
        if perturbed:
            sp = [s1[i] ^ gamma[i] for i in range(n)]
        elif settle_law:
            sp = self.rule_update(s1, lambda i: self.env_uniform(seed, e, step, 0, i))
        else:
            sp = self.rule_update(s1, lambda i: self.group_uniform(seed, G, b, step, i))
        # settle law (spec.settle >= 2): update k = 1.. from SETTLE_ENV gaps and the env's
        # SETTLE_SEL uniforms until sp is an attractor state, at most spec.settle updates in all
        unsettled = False
        for k in range(1, self.spec.settle):
            if tuple(sp) in self.att_of:
                break
            gk, pos, j = [0] * n, -1, 0
            while pos < n - 1:
                if j % 4 == 0:
                    P = draw(seed, e, step, SETTLE_ENV, ((k - 1) << 8) | (j // 4))
                pos += self.gap(P[j % 4])
                j += 1
                if pos >= n:
                    break
                gk[pos] = 1
            if any(gk):
                sp = [sp[i] ^ gk[i] for i in range(n)]
                perturbed = True
            else:
                sp = self.rule_update(sp, lambda i, k=k: self.env_uniform(seed, e, step, k, i))
        else:
            unsettled = self.spec.settle >= 2 and tuple(sp) not in self.att_of
        a = self.att_of.get(tuple(sp), -1)
        in_attr = a >= 0
        term = in_attr and a == target
        tt = min(t + 1, 255)
        trunc = self.spec.horizon > 0 and tt >= self.spec.horizon
        wrong = in_attr and not term
        reward = self.spec.reward_value(term, wrong, sum(flip))
        flags = int(term) | (int(trunc) << 1) | (int(in_attr) << 2) | (int(perturbed) << 3) | (int(unsettled) << 5)
        out = {"final_state": sp, "reward": reward, "flipmask": flip, "target": target}
        if (mode & MODE_AUTORESET) and (term or trunc):
            ns, tg = reset_to if reset_to is not None else self.random_state(seed, e, step)
            out.update(state_out=ns, target=tg, t=0, flags=flags | 16)
        else:
            out.update(state_out=sp, t=tt, flags=flags)
        return out
