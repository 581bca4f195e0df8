#!/bin/bash
# GPU session J (round 2): record-major LDS node records -- GPU tests, launch fits at 65,536 and
# 1,048,576 envs, LDS bank-conflict pass.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/j
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/j/gputest.log 2>&1 || { echo "GPU TESTS FAILED"; tail -60 gpurun_out/j/gputest.log; exit 1; }
tail -2 gpurun_out/j/gputest.log
for envs in 65536 1048576; do
  timeout -k 10 200 python tools/chunk_fit.py --envs $envs --steps 20,100 --reps 10 --mode eager --out gpurun_out/j/fit.jsonl > /dev/null || { echo "FIT $envs FAILED"; exit 1; }
done
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-trace --stats --output-format csv -d gpurun_out/j/pmc_a -o run -- python3 tools/chunk_fit.py --envs 1048576 --steps 20 --reps 5 --mode eager > gpurun_out/j/pmc_a.log 2>&1 || { echo "PMC FAILED"; exit 1; }
cat gpurun_out/j/fit.jsonl
