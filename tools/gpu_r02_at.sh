#!/bin/bash
# GPU session AT (round 2): the selection wave's raised priority re-measured on the Philox4x32-7
# build -- default (grids of at most four blocks per CU), never (sp0), always (sp1) -- at 65,536 to 1M
# envs (launch times of 20 and 100 steps), three reps; and the transposes' J = 16 stage (xv1) and J = 16, 4
# stages (xv2) on the VALU in place of ds_swizzle, with the parity tests on both.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/at
export TMPDIR=/tmp
for rep in 1 2 3; do
  for lib in libpbn_env_diag_base.so libpbn_env_sp0.so libpbn_env_sp1.so libpbn_env_xv1.so libpbn_env_xv2.so; do
    for envs in 65536 262144 1048576; do
      PBN_LIB=pbn_rl_amd/$lib timeout -k 10 120 python tools/chunk_fit.py --envs $envs --steps 20,100 --reps 10 --mode eager --out gpurun_out/at/$lib.jsonl > /dev/null || { echo "FIT $lib FAILED"; exit 1; }
    done
  done
done
for f in gpurun_out/at/*.jsonl; do echo $f; python -c "
import json
for l in open('$f'): d=json.loads(l); print(d['envs'], {k: round(v,2) for k,v in d['median_us'].items()})"; done
for lib in libpbn_env_xv1.so libpbn_env_xv2.so; do
  PBN_LIB=pbn_rl_amd/$lib timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/at/parity_$lib.log 2>&1 || { echo "PARITY $lib FAILED"; tail -30 gpurun_out/at/parity_$lib.log; exit 1; }
  tail -1 gpurun_out/at/parity_$lib.log
done
