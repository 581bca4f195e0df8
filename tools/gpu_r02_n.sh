#!/bin/bash
# GPU session N (round 2): the current product build end to end -- GPU tests, the driver's bench
# command, the 2000-step bench, config 5 (bdq), the driver command under the kernel trace, and the
# HBM-byte / SQ counter passes of 20- and 100-step launches (profiles/pmc_*_T*.json).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/n
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/n/gputest.log 2>&1 || { echo "GPU TESTS FAILED"; tail -60 gpurun_out/n/gputest.log; exit 1; }
tail -2 gpurun_out/n/gputest.log
for T in 20 100; do
  for pass in "fetch:FETCH_SIZE" "write:WRITE_SIZE" "sq:SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"; do
    name=${pass%%:*}; ctrs=${pass#*:}
    timeout -s KILL 120 rocprofv3 --pmc $ctrs --kernel-trace --stats --output-format csv -d gpurun_out/n/pmc/T${T}/pmc_$name -o run -- python3 tools/chunk_fit.py --steps $T --reps 10 --mode eager > gpurun_out/n/pmc_T${T}_$name.log 2>&1 || { echo "PMC $T $name FAILED"; exit 1; }
  done
done
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/n/bench_driver.json 2> gpurun_out/n/bench_driver.err || { echo BENCH FAILED; tail -20 gpurun_out/n/bench_driver.err; exit 1; }
tail -1 gpurun_out/n/bench_driver.json | cut -c1-300
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/n/bench_default.json 2> gpurun_out/n/bench_default.err || { echo BENCH2 FAILED; exit 1; }
timeout -k 10 300 python bench.py --workload bdq --cpu-seconds 5 > gpurun_out/n/bench_bdq.json 2> gpurun_out/n/bench_bdq.err || { echo BENCH3 FAILED; tail -20 gpurun_out/n/bench_bdq.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/n/prof_driver -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/n/prof_driver.log 2>&1 || { echo PROF FAILED; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/n/prof_bdq -o run -- python3 bench.py --workload bdq --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/n/prof_bdq.log 2>&1 || { echo PROF2 FAILED; exit 1; }
echo done
