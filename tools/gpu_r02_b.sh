#!/bin/bash
# GPU session B (round 2): GPU tests, the driver's bench command, and its kernel trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest.log 2>&1 || { echo "GPU TESTS FAILED"; tail -40 gpurun_out/gputest.log; exit 1; }
tail -3 gpurun_out/gputest.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_driver.json 2> gpurun_out/bench_driver.err || { echo BENCH1 FAILED; tail -20 gpurun_out/bench_driver.err; exit 1; }
cat gpurun_out/bench_driver.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_driver -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof_driver.log 2>&1 || { echo PROF FAILED; tail -20 gpurun_out/prof_driver.log; exit 1; }
echo done
