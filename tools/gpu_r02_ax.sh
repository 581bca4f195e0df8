#!/bin/bash
# GPU session AX (round 2): register budget of single-word states on the final build -- 4 and 5 waves per SIMD (we4, we5) against 6 (the product)
# at 65,536 and 1M envs, launches of 20 and 100 steps, three reps.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/ax
export TMPDIR=/tmp
for rep in 1 2 3; do
  for lib in libpbn_env_diag_base.so libpbn_env_we4.so libpbn_env_we5.so; do
    for envs in 65536 1048576; do
      PBN_LIB=pbn_rl_amd/$lib timeout -k 10 120 python tools/chunk_fit.py --envs $envs --steps 20,100 --reps 10 --mode eager --out gpurun_out/ax/$lib.jsonl > /dev/null || { echo "FIT $lib FAILED"; exit 1; }
    done
  done
done
echo ALL DONE
