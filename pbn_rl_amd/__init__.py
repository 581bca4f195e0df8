"""pbn_rl_amd -- MI355X-native batched PBN environment (gym-PBN step hot path).

Public surface:
  network.Network / load_network     ISPL + logic-function compiler
  attractors                         attractor fixtures / discovery
  spec.EnvSpec                       one environment definition (C descriptor)
  vector_env.VectorPBNEnv            batched envs in HBM, stepped by libpbn_env.so
  env.PBNEnv / make                  scalar gym-style facade (drop-in under train_BDQ.py)
"""
__version__ = "0.1.0"
