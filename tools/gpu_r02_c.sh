#!/bin/bash
# GPU session C (round 2): driver bench after the capture fix, its kernel trace, launch-length fit.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 3 > gpurun_out/bench_driver_c.json 2> gpurun_out/bench_driver_c.err || { echo BENCH FAILED; tail -20 gpurun_out/bench_driver_c.err; exit 1; }
cat gpurun_out/bench_driver_c.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_driver_c -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof_driver_c.log 2>&1 || { echo PROF FAILED; tail -20 gpurun_out/prof_driver_c.log; exit 1; }
timeout -k 10 300 python tools/chunk_fit.py --out gpurun_out/chunk_fit.jsonl || { echo FIT FAILED; exit 1; }
echo done
