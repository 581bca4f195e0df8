#!/bin/bash
# GPU session W (round 2): saddr output addressing (uniform per-step base + 32-bit lane offset), and
# the same with 6 waves per SIMD forced (diag_v1) -- GPU tests, then A/B launch fits against the
# HEAD build (diag_base).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/w
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/w/gputest.log 2>&1 || { echo "GPU TESTS FAILED"; tail -60 gpurun_out/w/gputest.log; exit 1; }
tail -2 gpurun_out/w/gputest.log
for rep in 1 2; do
for envs in 65536 1048576; do
  for lib in libpbn_env_diag_base.so libpbn_env_diag_v1.so libpbn_env.so; do
    PBN_LIB=pbn_rl_amd/$lib timeout -k 10 200 python tools/chunk_fit.py --envs $envs --steps 20,100 --reps 10 --mode eager --out gpurun_out/w/$lib.jsonl > /dev/null || { echo "FIT $lib $envs FAILED"; exit 1; }
  done
done
done
for f in gpurun_out/w/*.jsonl; do echo $f; python -c "
import json
for l in open('$f'): d=json.loads(l); print(d['envs'], round(d['fit_per_step_us'],3), d['median_us'])"; done
