#!/bin/bash
# GPU session A (round 2): tests, driver-shaped bench, default bench, kernel trace, probes.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
{ nproc; python -c "import os;print('affinity',len(os.sched_getaffinity(0)),'cpu_count',os.cpu_count())"; cat /sys/fs/cgroup/cpu.max 2>&1; echo OMP=$OMP_NUM_THREADS; } > gpurun_out/probe.txt 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gputest.log 2>&1 || { echo "GPU TESTS FAILED rc=$?"; tail -40 gpurun_out/gputest.log; exit 1; }
tail -3 gpurun_out/gputest.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_driver.json 2> gpurun_out/bench_driver.err || { echo BENCH1 FAILED; tail -20 gpurun_out/bench_driver.err; exit 1; }
cat gpurun_out/bench_driver.json
timeout -k 10 300 python bench.py --gpus 2 --steps 20 --warmup 5 > gpurun_out/bench_g2.out 2>&1; echo "gpus2 rc=$?" >> gpurun_out/probe.txt
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { echo BENCH2 FAILED; tail -20 gpurun_out/bench_default.err; exit 1; }
cat gpurun_out/bench_default.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_driver -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof_driver.log 2>&1 || { echo PROF FAILED; tail -20 gpurun_out/prof_driver.log; exit 1; }
timeout -k 10 300 python tools/gen_wide_attractors.py bb33 m47 > gpurun_out/wide_att.log 2>&1 || { echo WIDE FAILED; tail -20 gpurun_out/wide_att.log; }
cat gpurun_out/wide_att.log gpurun_out/probe.txt
