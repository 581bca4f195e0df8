#!/bin/bash
# GPU session AV (round 2): HEAD re-check -- GPU tests + smoke, and the two table rows still on
# older builds: 8,388,608 envs on one GPU and compute_ssd_hist at the reference's settings.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/av
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/av/gputest.log 2>&1 || { echo "GPU TESTS FAILED"; tail -60 gpurun_out/av/gputest.log; exit 1; }
tail -1 gpurun_out/av/gputest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/av/smoke.log 2>&1 || { echo "SMOKE FAILED"; cat gpurun_out/av/smoke.log; exit 1; }
grep smoke gpurun_out/av/smoke.log
timeout -k 10 300 python bench.py --envs 8388608 --steps 200 --warmup 100 --no-cpu-baseline --no-gather > gpurun_out/av/bench_8M.json 2> gpurun_out/av/bench_8M.err || { echo "8M FAILED"; tail gpurun_out/av/bench_8M.err; exit 1; }
echo "8M done"
timeout -k 10 300 python tools/ssd_bench.py > gpurun_out/av/ssd.json 2> gpurun_out/av/ssd.err || { echo "SSD FAILED"; tail gpurun_out/av/ssd.err; exit 1; }
echo ALL DONE
