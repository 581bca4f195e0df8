#!/bin/bash
# On the GPU box: bench line + rocprofv3 kernel stats + three PMC passes (FETCH_SIZE, WRITE_SIZE,
# SQ instruction counts with the VALU-busy / wave-state cycle counters and GRBM_GUI_ACTIVE)
# for the same bench command (the profiled passes without the hand-off passes, whose launches carry
# the own-shard copy: tools/handoff_trace.py attributes those).  Usage: tools/gpu_bench_profile.sh TAG [bench args...]
# Outputs under gpurun_out/TAG/.  Every GPU step has its own time limit; the first failure ends the script.
set -euo pipefail
tag=$1; shift
root=${GRAFT_REPO_ROOT:-/root/repo}
out=$root/gpurun_out/$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
cd "$root"
timeout -k 10 300 python bench.py "$@" > "$out/bench.json" 2> "$out/bench.err"
echo "bench done"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace" -o run -- \
  python bench.py --no-cpu-baseline --no-gather "$@" > "$out/trace_bench.json" 2> "$out/trace.err"
echo "trace done"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --stats --output-format csv -d "$out/pmc_fetch" -o run -- \
  python bench.py --no-cpu-baseline --no-gather "$@" > /dev/null 2> "$out/pmc_fetch.err"
echo "fetch done"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --stats --output-format csv -d "$out/pmc_write" -o run -- \
  python bench.py --no-cpu-baseline --no-gather "$@" > /dev/null 2> "$out/pmc_write.err"
echo "write done"
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES \
  SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --kernel-trace --stats \
  --output-format csv -d "$out/pmc_sq" -o run -- \
  python bench.py --no-cpu-baseline --no-gather "$@" > /dev/null 2> "$out/pmc_sq.err"
echo "sq done"
