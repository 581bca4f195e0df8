#!/bin/bash
# GPU session G (round 2): PMC passes (HBM bytes, SQ issue/wait breakdown) of 20- and 100-step
# pbn_rollout launches, pbn28 x 65,536 envs, one counter pass per run.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > gpurun_out/pmc/counters.txt 2>&1 || true
grep -c "SQ_" gpurun_out/pmc/counters.txt
for T in 20 100; do
  for pass in "fetch:FETCH_SIZE" "write:WRITE_SIZE" "sq:SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_BUSY_CYCLES"; do
    name=${pass%%:*}; ctrs=${pass#*:}
    timeout -s KILL 120 rocprofv3 --pmc $ctrs --kernel-trace --stats --output-format csv -d gpurun_out/pmc/T${T}/pmc_$name -o run -- python3 tools/chunk_fit.py --steps $T --reps 10 --mode eager > gpurun_out/pmc/T${T}_$name.log 2>&1 || { echo "PMC $T $name FAILED"; tail -5 gpurun_out/pmc/T${T}_$name.log; exit 1; }
  done
done
echo done
