#!/bin/bash
# GPU session AY (round 2): the selection wave's digit masks as one v_bfe per digit from per-lane thresholds in VGPRs (bfe) against the LDS mask table (the product)
# at 65,536 and 1M envs, launches of 20 and 100 steps, three reps.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/ay
export TMPDIR=/tmp
for rep in 1 2 3; do
  for lib in libpbn_env_diag_base.so libpbn_env_bfe.so; do
    for envs in 65536 1048576; do
      PBN_LIB=pbn_rl_amd/$lib timeout -k 10 120 python tools/chunk_fit.py --envs $envs --steps 20,100 --reps 10 --mode eager --out gpurun_out/ay/$lib.jsonl > /dev/null || { echo "FIT $lib FAILED"; exit 1; }
    done
  done
done
echo ALL DONE
PBN_LIB=pbn_rl_amd/libpbn_env_bfe.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ay/parity.log 2>&1 || { echo "PARITY FAILED"; tail -30 gpurun_out/ay/parity.log; exit 1; }
tail -1 gpurun_out/ay/parity.log
