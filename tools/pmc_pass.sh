#!/bin/bash
# Usage (on the GPU box): tools/pmc_pass.sh OUTDIR "COUNTERS" -- python tools/sweep.py ...
# One rocprofv3 counter pass (--pmc + --kernel-trace/--stats only, per the pool rules).
set -e
out=$1; shift
ctrs=$1; shift
shift  # --
cd /tmp && export TMPDIR=/tmp
exec_dir=${GRAFT_REPO_ROOT:-/root/repo}
cd "$exec_dir"
timeout -k 10 300 rocprofv3 --pmc $ctrs --kernel-trace --stats --output-format csv -d "$out" -o pmc -- "$@"
