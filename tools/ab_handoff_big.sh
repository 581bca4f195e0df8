#!/bin/bash
# A/B of the world-1 hand-off at 1M envs (pbn28, pbn70): pbn_rl_amd/libpbn_env_diag_g_burstbig.so, then this tree.
# Usage (on the GPU box): bash tools/ab_handoff_big.sh   (outputs under gpurun_out/r05_zj/)
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/r05_zj; mkdir -p $out
for side in burstbig tree; do
  if [ $side = tree ]; then unset PBN_LIB; else export PBN_LIB=$PWD/pbn_rl_amd/libpbn_env_diag_g_$side.so   # (a diagnostic build of the variant); fi
  for shape in "1m:--envs 1048576 --steps 500 --warmup 100" "pbn70:--network pbn70 --envs 1048576 --steps 200 --warmup 20"; do
    nm=${shape%%:*}; args=${shape#*:}
    timeout -k 10 300 python bench.py $args --no-cpu-baseline --settle-line 0 > $out/${side}_$nm.json 2> $out/${side}_$nm.err || { echo FAIL $side $nm; exit 1; }
    python -c "import json; d=[json.loads(l) for l in open('$out/${side}_$nm.json') if l.startswith('{')][-1]; print('$side $nm', d['value'], d['value_with_gather']/d['value'])"
  done
done
