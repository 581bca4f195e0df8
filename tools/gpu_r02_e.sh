#!/bin/bash
# GPU session E (round 2): GPU tests after the variant removal, launch-length fit graph vs eager.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest_e.log 2>&1 || { echo "GPU TESTS FAILED"; tail -60 gpurun_out/gputest_e.log; exit 1; }
tail -3 gpurun_out/gputest_e.log
timeout -k 10 300 python tools/chunk_fit.py --mode graph --out gpurun_out/chunk_fit_e.jsonl || { echo FIT FAILED; exit 1; }
timeout -k 10 300 python tools/chunk_fit.py --mode eager --out gpurun_out/chunk_fit_e.jsonl || { echo FIT FAILED; exit 1; }
echo done
