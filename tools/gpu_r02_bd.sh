#!/bin/bash
# GPU session BD (round 2): the selection wave with half its SEL calls (selhalf; results wrong, timing only), the upper bound of splitting the selection over two waves, against the product
# at 65,536 and 1M envs, launches of 20 and 100 steps, three reps.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/bd
export TMPDIR=/tmp
for rep in 1 2 3; do
  for lib in libpbn_env_diag_base.so libpbn_env_selhalf.so; do
    for envs in 65536 1048576; do
      PBN_LIB=pbn_rl_amd/$lib timeout -k 10 120 python tools/chunk_fit.py --envs $envs --steps 20,100 --reps 10 --mode eager --out gpurun_out/bd/$lib.jsonl > /dev/null || { echo "FIT $lib FAILED"; exit 1; }
    done
  done
done
echo ALL DONE
