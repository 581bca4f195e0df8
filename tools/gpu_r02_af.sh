#!/bin/bash
# GPU session AF (round 2): where the pipelined kernel's waves run (stamps build with HW_ID /
# XCC_ID per wave) and the per-role clocks, at 65,536 and 1M envs.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/af
export TMPDIR=/tmp
for n in 65536 1048576; do
  timeout -k 10 120 python tools/stamps.py --pipe --rollout 20 --envs $n > gpurun_out/af/stamps_$n.json 2> gpurun_out/af/stamps_$n.err || { echo "STAMPS $n FAILED"; tail -20 gpurun_out/af/stamps_$n.err; exit 1; }
done
cat gpurun_out/af/stamps_65536.json
