#!/bin/bash
# GPU session AN (round 2): which half of session AM's v1 cost the prologue -- v1a: table image
# loads all issued before the stores, one copy; v1b: the old copy loop from 16 copies; v1: both.
# Launch times against HEAD at 65,536 envs (1, 20, 100 steps), three reps.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/an
export TMPDIR=/tmp
for rep in 1 2 3; do
  for lib in libpbn_env_diag_base.so libpbn_env_v1a.so libpbn_env_v1b.so libpbn_env_v1.so; do
    PBN_LIB=pbn_rl_amd/$lib timeout -k 10 120 python tools/chunk_fit.py --envs 65536 --steps 1,20,100 --reps 10 --mode eager --out gpurun_out/an/$lib.jsonl > /dev/null || { echo "FIT $lib FAILED"; exit 1; }
  done
done
for f in gpurun_out/an/*.jsonl; do echo $f; python -c "
import json
for l in open('$f'): d=json.loads(l); print(d['envs'], {k: round(v,2) for k,v in d['median_us'].items()})"; done
