#!/bin/bash
# GPU session T (round 2): one ENV Philox call per env-step (autoreset draws and gap 2 from
# words 3:2 after the action draw; u2 as X * x_mult off the draw chain) -- GPU tests, then A/B
# launch fits against the HEAD build.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/t2
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t2/gputest.log 2>&1 || { echo "GPU TESTS FAILED"; tail -60 gpurun_out/t2/gputest.log; exit 1; }
tail -2 gpurun_out/t2/gputest.log
for rep in 1 2; do
for envs in 65536 1048576; do
  for lib in libpbn_env_diag_base.so libpbn_env.so; do
    PBN_LIB=pbn_rl_amd/$lib timeout -k 10 200 python tools/chunk_fit.py --envs $envs --steps 20,100 --reps 10 --mode eager --out gpurun_out/t2/$lib.jsonl > /dev/null || { echo "FIT $lib $envs FAILED"; exit 1; }
  done
done
done
for f in gpurun_out/t2/*.jsonl; do echo $f; python -c "
import json
for l in open('$f'): d=json.loads(l); print(d['envs'], round(d['fit_per_step_us'],3), d['median_us'])"; done
