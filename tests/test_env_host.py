"""Host-side bookkeeping of the gym facade (no GPU): the attractor-growth visit table stays
bounded (it grew without bound over a long training run)."""
from pbn_rl_amd.env import PBNEnv


def test_visit_table_is_bounded():
    env = PBNEnv.__new__(PBNEnv)
    env.visit_cap = 64
    env._visits = {k: (2 if k % 10 == 0 else 1) for k in range(100)}
    env._prune_visits()
    assert len(env._visits) <= 32 and all(c > 1 for c in env._visits.values())
    env._visits = {k: 2 for k in range(100)}
    env._prune_visits()
    assert len(env._visits) == 50 and min(env._visits) == 50   # the oldest half went
