#!/bin/bash
# GPU session BB (round 2): the learner frame (bench.py --workload bdq-learn) on the final build.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/bb
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --workload bdq-learn > gpurun_out/bb/bench_bdq_learn.json 2> gpurun_out/bb/bench_bdq_learn.err || { echo "bdq-learn FAILED"; tail gpurun_out/bb/bench_bdq_learn.err; exit 1; }
python -c "
import json
for l in open('gpurun_out/bb/bench_bdq_learn.json'):
    if l.startswith('{'): d=json.loads(l); print('%.3e' % d['value'], d['ms_per_step'])"
