#!/bin/bash
# GPU session AE (round 2): re-measure the current build -- GPU tests, the driver's bench command
# with kernel stats + PMC (tools/gpu_bench_profile.sh), the 2,000-step line, 1M envs and pbn70.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/ae
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ae/gputest.log 2>&1 || { echo "GPU TESTS FAILED"; tail -60 gpurun_out/ae/gputest.log; exit 1; }
tail -2 gpurun_out/ae/gputest.log
bash tools/gpu_bench_profile.sh ae/driver --gpus 1 --steps 20 --warmup 5 || { echo "DRIVER PROFILE FAILED"; exit 1; }
bash tools/gpu_bench_profile.sh ae/s2000 --gpus 1 --steps 2000 --warmup 200 || { echo "2000 PROFILE FAILED"; exit 1; }
timeout -k 10 300 python bench.py --envs 1048576 --steps 500 --warmup 100 --no-cpu-baseline > gpurun_out/ae/bench_1M.json 2> gpurun_out/ae/bench_1M.err || { echo "1M FAILED"; exit 1; }
timeout -k 10 300 python bench.py --network pbn70 --envs 1048576 --steps 200 --warmup 20 > gpurun_out/ae/bench_pbn70.json 2> gpurun_out/ae/bench_pbn70.err || { echo "pbn70 FAILED"; exit 1; }
echo ALL DONE
