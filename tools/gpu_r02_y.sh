#!/bin/bash
# GPU session Y (round 2): slot-major attractor hash (one LDS read per probe) + pc-major reward rows
# (diag_v1), plus the env wave computing the next step's ENV call (libpbn_env.so) -- GPU tests, then
# A/B launch fits against the HEAD build (diag_base).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/y
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/y/gputest.log 2>&1 || { echo "GPU TESTS FAILED"; tail -60 gpurun_out/y/gputest.log; exit 1; }
tail -2 gpurun_out/y/gputest.log
for rep in 1 2; do
for envs in 65536 1048576; do
  for lib in libpbn_env_diag_base.so libpbn_env_diag_v1.so libpbn_env.so; do
    PBN_LIB=pbn_rl_amd/$lib timeout -k 10 200 python tools/chunk_fit.py --envs $envs --steps 20,100 --reps 10 --mode eager --out gpurun_out/y/$lib.jsonl > /dev/null || { echo "FIT $lib $envs FAILED"; exit 1; }
  done
done
done
for f in gpurun_out/y/*.jsonl; do echo $f; python -c "
import json
for l in open('$f'): d=json.loads(l); print(d['envs'], round(d['fit_per_step_us'],3), d['median_us'])"; done
# pbn70 x 1M (config 3): 3-word states held to 3 waves per SIMD (libpbn_env.so) vs the compiler's
# 181 VGPRs (diag_v2)
for lib in libpbn_env_diag_v2.so libpbn_env.so; do
  PBN_LIB=pbn_rl_amd/$lib timeout -k 10 200 python tools/chunk_fit.py --network pbn70 --envs 1048576 --steps 20,100 --reps 5 --mode eager --out gpurun_out/y/pbn70_$lib.jsonl > /dev/null || { echo "FIT pbn70 $lib FAILED"; exit 1; }
done
for f in gpurun_out/y/pbn70_*.jsonl; do echo $f; python -c "
import json
for l in open('$f'): d=json.loads(l); print(d['envs'], round(d['fit_per_step_us'],3), d['median_us'])"; done
