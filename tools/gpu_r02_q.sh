#!/bin/bash
# GPU session Q (round 2): the other configs on the current build -- pbn70 x 1M (config 3),
# pbn28 x 1M (config 4's per-GPU shard), pbn28 x 8M, the SSD evaluation, and smoke().
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/q
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --network pbn70 --envs 1048576 --steps 200 --warmup 20 --cpu-seconds 5 > gpurun_out/q/bench_pbn70_1M.json 2> gpurun_out/q/e1.err || { echo B1 FAILED; tail -5 gpurun_out/q/e1.err; exit 1; }
timeout -k 10 300 python bench.py --envs 1048576 --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/q/bench_pbn28_1M.json 2> gpurun_out/q/e2.err || { echo B2 FAILED; exit 1; }
timeout -k 10 300 python bench.py --envs 8388608 --steps 200 --warmup 20 --no-cpu-baseline --no-gather > gpurun_out/q/bench_pbn28_8M.json 2> gpurun_out/q/e3.err || { echo B3 FAILED; tail -5 gpurun_out/q/e3.err; exit 1; }
timeout -k 10 300 python tools/ssd_bench.py > gpurun_out/q/ssd.json 2> gpurun_out/q/e4.err || { echo SSD FAILED; tail -5 gpurun_out/q/e4.err; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/q/smoke.log 2>&1 || { echo SMOKE FAILED; tail -5 gpurun_out/q/smoke.log; exit 1; }
for f in gpurun_out/q/bench_*.json; do tail -1 $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value'], d['ms_per_step'], d['roofline']['frac'], (d.get('cpu_baseline') or {}).get('value'))"; done
tail -2 gpurun_out/q/ssd.json; cat gpurun_out/q/smoke.log | tail -1
