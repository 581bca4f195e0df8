#!/bin/bash
# GPU session AS (round 2): final build (Philox4x32-7 streams, non-temporal output stores) -- GPU tests + smoke, the driver's bench command
# with kernel stats + PMC, the 2,000-step line, 1M envs, pbn70 and the BDQ frame (config 5).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/as
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/as/gputest.log 2>&1 || { echo "GPU TESTS FAILED"; tail -60 gpurun_out/as/gputest.log; exit 1; }
tail -2 gpurun_out/as/gputest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/as/smoke.log 2>&1 || { echo "SMOKE FAILED"; cat gpurun_out/as/smoke.log; exit 1; }
cat gpurun_out/as/smoke.log
bash tools/gpu_bench_profile.sh as/driver --gpus 1 --steps 20 --warmup 5 || { echo "DRIVER PROFILE FAILED"; exit 1; }
bash tools/gpu_bench_profile.sh as/s2000 --gpus 1 --steps 2000 --warmup 200 || { echo "2000 PROFILE FAILED"; exit 1; }
timeout -k 10 300 python bench.py --envs 1048576 --steps 500 --warmup 100 --no-cpu-baseline > gpurun_out/as/bench_1M.json 2> gpurun_out/as/bench_1M.err || { echo "1M FAILED"; exit 1; }
echo "1M done"
timeout -k 10 300 python bench.py --network pbn70 --envs 1048576 --steps 200 --warmup 20 > gpurun_out/as/bench_pbn70.json 2> gpurun_out/as/bench_pbn70.err || { echo "pbn70 FAILED"; exit 1; }
echo "pbn70 done"
timeout -k 10 300 python bench.py --workload bdq > gpurun_out/as/bench_bdq.json 2> gpurun_out/as/bench_bdq.err || { echo "bdq FAILED"; exit 1; }
echo ALL DONE
