#!/bin/bash
# GPU session V (round 2): per-role phase clocks (PBN_STAMPS builds) of the pipelined rollout,
# HEAD build (two ENV calls) vs the single-ENV-call build, 65,536 and 1M envs.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/v
export TMPDIR=/tmp
for envs in 65536 1048576; do
  for lib in libpbn_env_stamps_base.so libpbn_env_stamps.so; do
    timeout -k 10 120 python tools/stamps.py --pipe --rollout 20 --envs $envs --lib pbn_rl_amd/$lib > gpurun_out/v/${lib%.so}_$envs.json 2> gpurun_out/v/err.log || { echo "STAMPS $lib $envs FAILED"; tail -5 gpurun_out/v/err.log; exit 1; }
  done
done
for f in gpurun_out/v/*.json; do echo $f; python -c "import json; d=json.load(open('$f')); print({k: d[k] for k in d if k not in ('envs','blocks','rollout_steps')})"; done
