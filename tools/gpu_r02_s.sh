#!/bin/bash
# GPU session S (round 2): per-role step loops, swizzle/perm transposes, padded node chain with
# byte-offset gathers -- GPU tests, then A/B launch fits: HEAD build (diag_base), per-role loops
# alone (diag_v1), all three (libpbn_env.so).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/s
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s/gputest.log 2>&1 || { echo "GPU TESTS FAILED"; tail -60 gpurun_out/s/gputest.log; exit 1; }
tail -2 gpurun_out/s/gputest.log
for rep in 1 2; do
for envs in 65536 1048576; do
  for lib in libpbn_env_diag_base.so libpbn_env_diag_v1.so libpbn_env.so; do
    PBN_LIB=pbn_rl_amd/$lib timeout -k 10 200 python tools/chunk_fit.py --envs $envs --steps 20,100 --reps 10 --mode eager --out gpurun_out/s/$lib.jsonl > /dev/null || { echo "FIT $lib $envs FAILED"; exit 1; }
  done
done
done
for f in gpurun_out/s/*.jsonl; do echo $f; python -c "
import json
for l in open('$f'): d=json.loads(l); print(d['envs'], round(d['fit_per_step_us'],3), d['median_us'])"; done
