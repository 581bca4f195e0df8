#!/bin/bash
# GPU session AG (round 2): wave-priority variants of the pipelined kernel (diagnostic builds
# libpbn_env_v1..v4: env prio 1, env prio 2, state 3 + env 2, selection prio 1) against HEAD,
# interleaved, two reps: launch fits at 65,536 and 1M envs.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/ah
export TMPDIR=/tmp
for rep in 1 2; do
  for lib in libpbn_env.so libpbn_env_v1.so libpbn_env_v2.so libpbn_env_v3.so libpbn_env_v4.so libpbn_env_v5.so; do
    PBN_LIB=pbn_rl_amd/$lib timeout -k 10 120 python tools/chunk_fit.py --envs 65536 --steps 20,100 --reps 10 --mode eager --out gpurun_out/ah/$lib.jsonl > /dev/null || { echo "FIT $lib FAILED"; exit 1; }
    PBN_LIB=pbn_rl_amd/$lib timeout -k 10 120 python tools/chunk_fit.py --envs 262144 --steps 100 --reps 5 --out gpurun_out/ah/$lib.jsonl > /dev/null && PBN_LIB=pbn_rl_amd/$lib timeout -k 10 120 python tools/chunk_fit.py --envs 1048576 --steps 100 --reps 5 --mode eager --out gpurun_out/ah/$lib.jsonl > /dev/null || { echo "FIT $lib FAILED"; exit 1; }
  done
done
for f in gpurun_out/ah/*.jsonl; do echo $f; python -c "
import json
for l in open('$f'): d=json.loads(l); print(d['envs'], {k: round(v,2) for k,v in d['median_us'].items()})"; done
