#!/bin/bash
# GPU session AM (round 2): launch prologue -- v1: the table image read once per thread (all
# loads before the stores) from one of 16 copies per XCD; v2 (libpbn_env.so): v1 + step 0's
# Philox words computed while the image is in flight.  GPU tests, launch times against HEAD at
# 65,536 (1, 20, 100 steps) and 1M envs, three reps, and the stamps build's launch anatomy.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/am
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/am/gputest.log 2>&1 || { echo "GPU TESTS FAILED"; tail -60 gpurun_out/am/gputest.log; exit 1; }
tail -2 gpurun_out/am/gputest.log
for rep in 1 2 3; do
  for lib in libpbn_env_diag_base.so libpbn_env_v1.so libpbn_env.so; do
    PBN_LIB=pbn_rl_amd/$lib timeout -k 10 120 python tools/chunk_fit.py --envs 65536 --steps 1,20,100 --reps 10 --mode eager --out gpurun_out/am/$lib.jsonl > /dev/null || { echo "FIT $lib FAILED"; exit 1; }
    PBN_LIB=pbn_rl_amd/$lib timeout -k 10 120 python tools/chunk_fit.py --envs 1048576 --steps 100 --reps 5 --mode eager --out gpurun_out/am/$lib.jsonl > /dev/null || { echo "FIT $lib FAILED"; exit 1; }
  done
done
timeout -k 10 120 python tools/stamps.py --pipe --rollout 20 --envs 65536 > gpurun_out/am/stamps_65536_20.json 2> gpurun_out/am/stamps.err || { echo "STAMPS FAILED"; exit 1; }
for f in gpurun_out/am/*.jsonl; do echo $f; python -c "
import json
for l in open('$f'): d=json.loads(l); print(d['envs'], {k: round(v,2) for k,v in d['median_us'].items()})"; done
python -c "import json; d=json.load(open('gpurun_out/am/stamps_65536_20.json'))['anatomy']; d.pop('by_xcc'); print(json.dumps(d))"
