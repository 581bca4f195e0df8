#!/bin/bash
# GPU session M (round 2): A/B of hoisted S-plane gather addresses (diag_hoist) against the
# current build (diag_base); rollout parity of the hoisted build.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/m
export TMPDIR=/tmp
PBN_LIB=pbn_rl_amd/libpbn_env_diag_hoist.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k rollout -x -q --timeout 300 --timeout-method thread > gpurun_out/m/parity.log 2>&1 || { echo "PARITY FAILED"; tail -40 gpurun_out/m/parity.log; exit 1; }
tail -1 gpurun_out/m/parity.log
for rep in 1 2; do
for envs in 65536 1048576; do
  for lib in libpbn_env_diag_base.so libpbn_env_diag_hoist.so; do
    PBN_LIB=pbn_rl_amd/$lib timeout -k 10 200 python tools/chunk_fit.py --envs $envs --steps 20,100 --reps 10 --mode eager --out gpurun_out/m/$lib.jsonl > /dev/null || { echo "FIT $lib $envs FAILED"; exit 1; }
  done
done
done
for f in gpurun_out/m/*.jsonl; do echo $f; python -c "
import json
for l in open('$f'): d=json.loads(l); print(d['envs'], round(d['fit_per_step_us'],3), d['median_us'])"; done
