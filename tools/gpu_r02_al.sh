#!/bin/bash
# GPU session AL (round 2): launch anatomy of the pipelined kernel (stamps build, state waves'
# s_memrealtime at entry / image / loop start / iterations 0, 1 / loop end / stores landed).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/al
export TMPDIR=/tmp
for cfg in "65536 20" "65536 100" "1048576 20"; do
  set -- $cfg
  timeout -k 10 120 python tools/stamps.py --pipe --rollout $2 --envs $1 > gpurun_out/al/stamps_$1_$2.json 2> gpurun_out/al/stamps_$1_$2.err || { echo "STAMPS $cfg FAILED"; tail -20 gpurun_out/al/stamps_$1_$2.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/al/stamps_$1_$2.json')); print('$cfg', d['iteration_median'], json.dumps(d['anatomy']))"
done
