#!/bin/bash
# GPU session AR (round 2): launch prologue -- non-temporal output stores (v1x) and the digit-mask
# table built beside the image copy (vx1), against neither (v00), at 65,536 and 1M envs
# (launch times of 20 and 100 steps), three reps; then the parity tests on the combined build.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/ar
export TMPDIR=/tmp
for rep in 1 2 3; do
  for lib in libpbn_env_v00.so libpbn_env_v10.so libpbn_env_v01.so libpbn_env_v11.so; do
    for envs in 65536 1048576; do
      PBN_LIB=pbn_rl_amd/$lib timeout -k 10 120 python tools/chunk_fit.py --envs $envs --steps 20,100 --reps 10 --mode eager --out gpurun_out/ar/$lib.jsonl > /dev/null || { echo "FIT $lib FAILED"; exit 1; }
    done
  done
done
for f in gpurun_out/ar/*.jsonl; do echo $f; python -c "
import json
for l in open('$f'): d=json.loads(l); print(d['envs'], {k: round(v,2) for k,v in d['median_us'].items()})"; done
PBN_LIB=pbn_rl_amd/libpbn_env_v11.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ar/parity.log 2>&1 || { echo "PARITY FAILED"; tail -30 gpurun_out/ar/parity.log; exit 1; }
tail -1 gpurun_out/ar/parity.log
