#!/bin/bash
# GPU session AP (round 2): the Philox round count's share at HEAD -- diagnostic builds with 7 and
# 8 rounds against the product (10) at 65,536 and 1M envs (launch times of 20 and 100 steps).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/ap
export TMPDIR=/tmp
for rep in 1 2; do
  for lib in libpbn_env_diag_base.so libpbn_env_r7.so libpbn_env_r8.so; do
    for envs in 65536 1048576; do
      PBN_LIB=pbn_rl_amd/$lib timeout -k 10 120 python tools/chunk_fit.py --envs $envs --steps 20,100 --reps 10 --mode eager --out gpurun_out/ap/$lib.jsonl > /dev/null || { echo "FIT $lib FAILED"; exit 1; }
    done
  done
done
for f in gpurun_out/ap/*.jsonl; do echo $f; python -c "
import json
for l in open('$f'): d=json.loads(l); print(d['envs'], {k: round(v,2) for k,v in d['median_us'].items()})"; done
