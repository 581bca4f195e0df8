#!/bin/bash
# GPU session Z (round 2): launch prologue -- LDS image copy with four loads in flight per thread,
# state loads issued before it, threshold digit masks built two threads per record -- GPU tests,
# then launch fits (1..100 steps) against the HEAD build.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/z
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/z/gputest.log 2>&1 || { echo "GPU TESTS FAILED"; tail -60 gpurun_out/z/gputest.log; exit 1; }
tail -2 gpurun_out/z/gputest.log
for rep in 1 2; do
  for lib in libpbn_env_diag_base.so libpbn_env.so; do
    PBN_LIB=pbn_rl_amd/$lib timeout -k 10 200 python tools/chunk_fit.py --envs 65536 --steps 1,2,5,20,100 --reps 10 --mode eager --out gpurun_out/z/$lib.jsonl > /dev/null || { echo "FIT $lib FAILED"; exit 1; }
    PBN_LIB=pbn_rl_amd/$lib timeout -k 10 200 python tools/chunk_fit.py --envs 1048576 --steps 20,100 --reps 5 --mode eager --out gpurun_out/z/$lib.jsonl > /dev/null || { echo "FIT $lib FAILED"; exit 1; }
  done
done
for f in gpurun_out/z/*.jsonl; do echo $f; python -c "
import json
for l in open('$f'): d=json.loads(l); print(d['envs'], round(d['fit_per_step_us'],3), round(d['fit_fixed_us'],2), round(d['tiny_kernel_us'],2), {k: round(v,2) for k,v in d['median_us'].items()})"; done
