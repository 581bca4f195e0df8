#!/bin/bash
# GPU session D (round 2): GPU tests (incl. the agent law pin), driver bench, launch-length fit.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest_d.log 2>&1 || { echo "GPU TESTS FAILED"; tail -60 gpurun_out/gputest_d.log; exit 1; }
tail -3 gpurun_out/gputest_d.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 3 > gpurun_out/bench_driver_d.json 2> gpurun_out/bench_driver_d.err || { echo BENCH FAILED; tail -20 gpurun_out/bench_driver_d.err; exit 1; }
tail -1 gpurun_out/bench_driver_d.json
timeout -k 10 300 python tools/chunk_fit.py --out gpurun_out/chunk_fit_d.jsonl || { echo FIT FAILED; exit 1; }
echo done
