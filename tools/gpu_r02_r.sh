#!/bin/bash
# GPU session R (round 2): validation of the committed build -- the GPU suite, the driver's
# bench command (traffic from the T20 PMC summary) and smoke().
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r/tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/r/tests.log; exit 1; }
tail -3 gpurun_out/r/tests.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r/bench_driver.json 2> gpurun_out/r/e1.err || { echo B1 FAILED; tail -5 gpurun_out/r/e1.err; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r/smoke.log 2>&1 || { echo SMOKE FAILED; tail -5 gpurun_out/r/smoke.log; exit 1; }
tail -1 gpurun_out/r/bench_driver.json; tail -1 gpurun_out/r/smoke.log
