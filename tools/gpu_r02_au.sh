#!/bin/bash
# GPU session AU (round 2): the fused BDQ tail (pbn_bdq_tail) -- agent tests, the whole GPU
# suite, the config 5 bench line with its kernel trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/au
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_agent.py -x -q --timeout 120 --timeout-method thread > gpurun_out/au/agent.log 2>&1 || { echo "AGENT TESTS FAILED"; tail -60 gpurun_out/au/agent.log; exit 1; }
tail -1 gpurun_out/au/agent.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/au/gputest.log 2>&1 || { echo "GPU TESTS FAILED"; tail -60 gpurun_out/au/gputest.log; exit 1; }
tail -1 gpurun_out/au/gputest.log
timeout -k 10 300 python bench.py --workload bdq > gpurun_out/au/bench_bdq.json 2> gpurun_out/au/bench_bdq.err || { echo "bdq FAILED"; tail gpurun_out/au/bench_bdq.err; exit 1; }
echo "bdq done"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/au/trace_bdq -o run -- python bench.py --workload bdq --no-cpu-baseline > gpurun_out/au/trace_bdq.json 2> gpurun_out/au/trace_bdq.err || { echo "bdq trace FAILED"; exit 1; }
echo ALL DONE
