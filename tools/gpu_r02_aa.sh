#!/bin/bash
# GPU session AA (round 2): role shares of the current pipelined kernel -- diagnostic builds with
# one role's work removed (PBN_DIAG_SKIP_ROLE = 0 state, 1 env draws, 2 selection; results
# wrong, timing only) against the product, 65,536 and 1M envs.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/aa2
export TMPDIR=/tmp
for envs in 65536 1048576; do
  for lib in libpbn_env.so libpbn_env_diag_skip0.so libpbn_env_diag_skip1.so libpbn_env_diag_skip2.so; do
    PBN_LIB=pbn_rl_amd/$lib timeout -k 10 200 python tools/chunk_fit.py --envs $envs --steps 20,100 --reps 8 --mode eager --out gpurun_out/aa2/$lib.jsonl > /dev/null || { echo "FIT $lib $envs FAILED"; exit 1; }
  done
done
for f in gpurun_out/aa2/*.jsonl; do echo $f; python -c "
import json
for l in open('$f'): d=json.loads(l); print(d['envs'], round(d['fit_per_step_us'],3), {k: round(v,2) for k,v in d['median_us'].items()})"; done
