#!/bin/bash
# GPU session H (round 2): the RNG's share of the rollout kernel -- launch-length fit with the
# product library and with diagnostic builds running 2 and 6 Philox rounds (wrong results,
# timing only), at 65,536 and 1,048,576 envs.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for envs in 65536 1048576; do
  for lib in libpbn_env.so libpbn_env_diag_r6.so libpbn_env_diag_r2.so; do
    PBN_LIB=pbn_rl_amd/$lib timeout -k 10 200 python tools/chunk_fit.py --envs $envs --steps 20,100 --reps 10 --mode eager --out gpurun_out/rounds_$lib.jsonl > /dev/null || { echo "FIT $lib $envs FAILED"; exit 1; }
  done
done
cat gpurun_out/rounds_*.jsonl
