#!/bin/bash
# GPU session U (round 2): SQ counters per launch (VALU / SALU / LDS instructions, wave and busy
# cycles) of the HEAD build and the single-ENV-call build, pbn28 x 1M and x 65,536, 100 steps.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/u
export TMPDIR=/tmp
C="SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
for envs in 1048576 65536; do
  for lib in libpbn_env_diag_base.so libpbn_env.so; do
    PBN_LIB=pbn_rl_amd/$lib bash tools/pmc_pass.sh gpurun_out/u/${lib%.so}_$envs "$C" -- python3 tools/chunk_fit.py --envs $envs --steps 100 --reps 3 --mode eager > /dev/null 2>&1 || { echo "PMC $lib $envs FAILED"; exit 1; }
  done
done
ls gpurun_out/u/*/
