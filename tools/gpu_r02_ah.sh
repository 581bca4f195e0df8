#!/bin/bash
# GPU session AH (round 2): wave-priority orders (state, env, selection) of the pipelined kernel,
# diagnostic builds v1 = 3 2 1, v2 = 2 1 1, v3 = 3 1 2, v4 = 2 0 2, v5 = 2 0 1 against HEAD (2 0 0),
# interleaved, two reps: launch times at 65,536, 262,144 and 1M envs.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/ah
export TMPDIR=/tmp
for rep in 1 2; do
  for lib in libpbn_env.so libpbn_env_v1.so libpbn_env_v2.so libpbn_env_v3.so libpbn_env_v4.so libpbn_env_v5.so; do
    PBN_LIB=pbn_rl_amd/$lib timeout -k 10 120 python tools/chunk_fit.py --envs 65536 --steps 20,100 --reps 10 --mode eager --out gpurun_out/ah/$lib.jsonl > /dev/null || { echo "FIT $lib FAILED"; exit 1; }
    PBN_LIB=pbn_rl_amd/$lib timeout -k 10 120 python tools/chunk_fit.py --envs 262144 --steps 100 --reps 5 --mode eager --out gpurun_out/ah/$lib.jsonl > /dev/null && PBN_LIB=pbn_rl_amd/$lib timeout -k 10 120 python tools/chunk_fit.py --envs 1048576 --steps 100 --reps 5 --mode eager --out gpurun_out/ah/$lib.jsonl > /dev/null || { echo "FIT $lib FAILED"; exit 1; }
  done
done
for f in gpurun_out/ah/*.jsonl; do echo $f; python -c "
import json
for l in open('$f'): d=json.loads(l); print(d['envs'], {k: round(v,2) for k,v in d['median_us'].items()})"; done
