#!/bin/bash
# GPU session AW (round 2): role shares on the final build -- diagnostic builds with one wave
# idle (skip0 = state, skip1 = env draws, skip2 = selection; results wrong, timing only) against
# the product, 65,536 and 1M envs, launches of 20 and 100 steps, three reps.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/aw
export TMPDIR=/tmp
for rep in 1 2 3; do
  for lib in libpbn_env_diag_base.so libpbn_env_skip0.so libpbn_env_skip1.so libpbn_env_skip2.so; do
    for envs in 65536 1048576; do
      PBN_LIB=pbn_rl_amd/$lib timeout -k 10 120 python tools/chunk_fit.py --envs $envs --steps 20,100 --reps 10 --mode eager --out gpurun_out/aw/$lib.jsonl > /dev/null || { echo "FIT $lib FAILED"; exit 1; }
    done
  done
done
echo ALL DONE
