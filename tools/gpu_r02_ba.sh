#!/bin/bash
# GPU session BA (round 2): the driver's exact bench command five times on one box (spread of
# the headline), final build.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/ba
export TMPDIR=/tmp
for r in 1 2 3 4 5; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/ba/bench_$r.json 2> gpurun_out/ba/bench_$r.err || { echo "BENCH $r FAILED"; tail gpurun_out/ba/bench_$r.err; exit 1; }
  python -c "
import json
for l in open('gpurun_out/ba/bench_$r.json'):
    if l.startswith('{'): d=json.loads(l); print($r, '%.3e' % d['value'], d['roofline']['launch_ms'], d['timing']['event_floor_us'])"
done
