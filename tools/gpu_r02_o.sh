#!/bin/bash
# GPU session O (round 2): per-role shares -- launch fits and SQ_INSTS_VALU of diagnostic builds in
# which one role of the pipelined kernel does no work; then the driver-shaped bench with the
# committed PMC summaries in place.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/o
export TMPDIR=/tmp
for lib in libpbn_env.so libpbn_env_diag_skip0.so libpbn_env_diag_skip1.so libpbn_env_diag_skip2.so; do
  PBN_LIB=pbn_rl_amd/$lib timeout -k 10 200 python tools/chunk_fit.py --envs 65536 --steps 20,100 --reps 10 --mode eager --out gpurun_out/o/fit_$lib.jsonl > /dev/null || { echo "FIT $lib FAILED"; exit 1; }
  PBN_LIB=pbn_rl_amd/$lib timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES --kernel-trace --stats --output-format csv -d gpurun_out/o/pmc_$lib -o run -- python3 tools/chunk_fit.py --envs 65536 --steps 100 --reps 5 --mode eager > gpurun_out/o/pmc_$lib.log 2>&1 || { echo "PMC $lib FAILED"; exit 1; }
done
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 3 > gpurun_out/o/bench_driver.json 2> gpurun_out/o/bench_driver.err || { echo BENCH FAILED; exit 1; }
tail -1 gpurun_out/o/bench_driver.json | cut -c1-600
echo done
