#!/bin/bash
# GPU session I (round 2): instruction mix and LDS behaviour of the rollout kernel at 65,536 and
# 1,048,576 envs (two SQ counter passes each, 20-step launches).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/pmc2
export TMPDIR=/tmp
for envs in 65536 1048576; do
  for pass in "a:SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "b:SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_INT64 SQ_INSTS_BRANCH SQ_LDS_ADDR_CONFLICT SQ_ACTIVE_INST_SCA"; do
    name=${pass%%:*}; ctrs=${pass#*:}
    timeout -s KILL 120 rocprofv3 --pmc $ctrs --kernel-trace --stats --output-format csv -d gpurun_out/pmc2/E${envs}/pmc_$name -o run -- python3 tools/chunk_fit.py --envs $envs --steps 20 --reps 5 --mode eager > gpurun_out/pmc2/E${envs}_$name.log 2>&1 || { echo "PMC $envs $name FAILED"; tail -5 gpurun_out/pmc2/E${envs}_$name.log; exit 1; }
  done
done
echo done
