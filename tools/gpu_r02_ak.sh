#!/bin/bash
# GPU session AK (round 2): the selection wave's last SEL call computed by the env-draw wave, one step ahead
# (LDS hand-off) -- GPU tests, then launch times against the HEAD build, three reps.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/ak
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ak/gputest.log 2>&1 || { echo "GPU TESTS FAILED"; tail -60 gpurun_out/ak/gputest.log; exit 1; }
tail -2 gpurun_out/ak/gputest.log
for rep in 1 2 3; do
  for lib in libpbn_env_diag_base.so libpbn_env.so; do
    PBN_LIB=pbn_rl_amd/$lib timeout -k 10 120 python tools/chunk_fit.py --envs 65536 --steps 20,100 --reps 10 --mode eager --out gpurun_out/ak/$lib.jsonl > /dev/null || { echo "FIT $lib FAILED"; exit 1; }
    PBN_LIB=pbn_rl_amd/$lib timeout -k 10 120 python tools/chunk_fit.py --envs 131072 --steps 100 --reps 5 --mode eager --out gpurun_out/ak/$lib.jsonl > /dev/null || { echo "FIT $lib FAILED"; exit 1; }
    PBN_LIB=pbn_rl_amd/$lib timeout -k 10 120 python tools/chunk_fit.py --envs 1048576 --steps 100 --reps 5 --mode eager --out gpurun_out/ak/$lib.jsonl > /dev/null || { echo "FIT $lib FAILED"; exit 1; }
  done
done
for f in gpurun_out/ak/*.jsonl; do echo $f; python -c "
import json
for l in open('$f'): d=json.loads(l); print(d['envs'], {k: round(v,2) for k,v in d['median_us'].items()})"; done
