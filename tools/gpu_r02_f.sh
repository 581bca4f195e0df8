#!/bin/bash
# GPU session F (round 2): GPU tests after the RNG re-freeze, driver bench (eager), its kernel trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest_f.log 2>&1 || { echo "GPU TESTS FAILED"; tail -60 gpurun_out/gputest_f.log; exit 1; }
tail -3 gpurun_out/gputest_f.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 3 > gpurun_out/bench_driver_f.json 2> gpurun_out/bench_driver_f.err || { echo BENCH FAILED; tail -20 gpurun_out/bench_driver_f.err; exit 1; }
tail -1 gpurun_out/bench_driver_f.json
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_default_f.json 2> gpurun_out/bench_default_f.err || { echo BENCH2 FAILED; tail -20 gpurun_out/bench_default_f.err; exit 1; }
tail -1 gpurun_out/bench_default_f.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_driver_f -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof_driver_f.log 2>&1 || { echo PROF FAILED; tail -20 gpurun_out/prof_driver_f.log; exit 1; }
echo done
