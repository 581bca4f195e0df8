#!/bin/bash
# GPU session AJ (round 2): env fast-path trims (guard-free action and gap bits, two steps per trip)
# + selection priority -- GPU tests, then launch times against the HEAD build, three reps.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/aj
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/aj/gputest.log 2>&1 || { echo "GPU TESTS FAILED"; tail -60 gpurun_out/aj/gputest.log; exit 1; }
tail -2 gpurun_out/aj/gputest.log
for rep in 1 2 3; do
  for lib in libpbn_env_diag_base.so libpbn_env.so; do
    PBN_LIB=pbn_rl_amd/$lib timeout -k 10 120 python tools/chunk_fit.py --envs 65536 --steps 20,100 --reps 10 --mode eager --out gpurun_out/aj/$lib.jsonl > /dev/null || { echo "FIT $lib FAILED"; exit 1; }
    PBN_LIB=pbn_rl_amd/$lib timeout -k 10 120 python tools/chunk_fit.py --envs 131072 --steps 100 --reps 5 --mode eager --out gpurun_out/aj/$lib.jsonl > /dev/null || { echo "FIT $lib FAILED"; exit 1; }
    PBN_LIB=pbn_rl_amd/$lib timeout -k 10 120 python tools/chunk_fit.py --envs 1048576 --steps 100 --reps 5 --mode eager --out gpurun_out/aj/$lib.jsonl > /dev/null || { echo "FIT $lib FAILED"; exit 1; }
  done
done
for f in gpurun_out/aj/*.jsonl; do echo $f; python -c "
import json
for l in open('$f'): d=json.loads(l); print(d['envs'], {k: round(v,2) for k,v in d['median_us'].items()})"; done
