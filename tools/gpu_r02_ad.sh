#!/bin/bash
# GPU session AD (round 2): state wave fast path (single-word states: record inputs in VGPRs, the
# step's selection masks and selectors read before the transpose) -- GPU tests, then launch fits
# against the HEAD build.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/ad
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ad/gputest.log 2>&1 || { echo "GPU TESTS FAILED"; tail -60 gpurun_out/ad/gputest.log; exit 1; }
tail -2 gpurun_out/ad/gputest.log
for rep in 1 2; do
  for lib in libpbn_env_diag_base.so libpbn_env.so; do
    PBN_LIB=pbn_rl_amd/$lib timeout -k 10 200 python tools/chunk_fit.py --envs 65536 --steps 1,2,5,20,100 --reps 10 --mode eager --out gpurun_out/ad/$lib.jsonl > /dev/null || { echo "FIT $lib FAILED"; exit 1; }
    PBN_LIB=pbn_rl_amd/$lib timeout -k 10 200 python tools/chunk_fit.py --envs 1048576 --steps 20,100 --reps 5 --mode eager --out gpurun_out/ad/$lib.jsonl > /dev/null || { echo "FIT $lib FAILED"; exit 1; }
  done
done
for f in gpurun_out/ad/*.jsonl; do echo $f; python -c "
import json
for l in open('$f'): d=json.loads(l); print(d['envs'], round(d['fit_per_step_us'],3), round(d['fit_fixed_us'],2), round(d['tiny_kernel_us'],2), {k: round(v,2) for k,v in d['median_us'].items()})"; done
