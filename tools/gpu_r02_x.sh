#!/bin/bash
# GPU session X (round 2): waves per SIMD forced to 6 / 7 / 8 (diag_v1 / v2 / v3: 80 / 72 / 64
# VGPRs, the last two with scratch spills in the state loop) -- A/B launch fits at 1M and 65,536.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/x
export TMPDIR=/tmp
for rep in 1 2; do
for envs in 1048576 65536; do
  for lib in libpbn_env_diag_v1.so libpbn_env_diag_v2.so libpbn_env_diag_v3.so; do
    PBN_LIB=pbn_rl_amd/$lib timeout -k 10 200 python tools/chunk_fit.py --envs $envs --steps 20,100 --reps 10 --mode eager --out gpurun_out/x/$lib.jsonl > /dev/null || { echo "FIT $lib $envs FAILED"; exit 1; }
  done
done
done
for f in gpurun_out/x/*.jsonl; do echo $f; python -c "
import json
for l in open('$f'): d=json.loads(l); print(d['envs'], round(d['fit_per_step_us'],3), d['median_us'])"; done
