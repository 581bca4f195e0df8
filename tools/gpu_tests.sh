#!/bin/bash
# On the GPU box: the -m gpu suite and smoke(), each under its own time limit.
# Usage: tools/gpu_tests.sh TAG [pytest selection...]   (outputs under gpurun_out/TAG/)
set -o pipefail
tag=$1; shift
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
sel=${*:-tests}
timeout -k 10 1000 python -u -m pytest $sel -m gpu -x -v --timeout 240 --timeout-method thread \
  > "$out/gputest.log" 2>&1 || { echo "GPU TESTS FAILED"; tail -60 "$out/gputest.log"; exit 1; }
tail -3 "$out/gputest.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1 \
  || { echo "SMOKE FAILED"; cat "$out/smoke.log"; exit 1; }
cat "$out/smoke.log"
