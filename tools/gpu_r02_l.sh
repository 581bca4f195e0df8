#!/bin/bash
# GPU session L (round 2): gap bucket table + lean transposes + single-state reset path:
# GPU tests, A/B launch fits against the previous build, VALU count pass.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/l
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/l/gputest.log 2>&1 || { echo "GPU TESTS FAILED"; tail -60 gpurun_out/l/gputest.log; exit 1; }
tail -2 gpurun_out/l/gputest.log
for rep in 1 2; do
for envs in 65536 1048576; do
  for lib in libpbn_env_diag_base.so libpbn_env.so; do
    PBN_LIB=pbn_rl_amd/$lib timeout -k 10 200 python tools/chunk_fit.py --envs $envs --steps 20,100 --reps 10 --mode eager --out gpurun_out/l/$lib.jsonl > /dev/null || { echo "FIT $lib $envs FAILED"; exit 1; }
  done
done
done
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY --kernel-trace --stats --output-format csv -d gpurun_out/l/pmc_sq -o run -- python3 tools/chunk_fit.py --envs 65536 --steps 100 --reps 5 --mode eager > gpurun_out/l/pmc.log 2>&1 || { echo "PMC FAILED"; exit 1; }
for f in gpurun_out/l/*.jsonl; do echo $f; python -c "
import json
for l in open('$f'): d=json.loads(l); print(d['envs'], round(d['fit_per_step_us'],3), d['median_us'])"; done
