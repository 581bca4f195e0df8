#!/bin/bash
# GPU session AO (round 2, re-entry): GPU tests + smoke at HEAD, the driver's bench command with
# kernel stats + PMC.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/ao
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ao/gputest.log 2>&1 || { echo "GPU TESTS FAILED"; tail -60 gpurun_out/ao/gputest.log; exit 1; }
tail -2 gpurun_out/ao/gputest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/ao/smoke.log 2>&1 || { echo "SMOKE FAILED"; cat gpurun_out/ao/smoke.log; exit 1; }
cat gpurun_out/ao/smoke.log
bash tools/gpu_bench_profile.sh ao/driver --gpus 1 --steps 20 --warmup 5 || { echo "DRIVER PROFILE FAILED"; exit 1; }
echo ALL DONE
