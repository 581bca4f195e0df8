set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r03_c
timeout -k 10 300 python -u -m pytest tests/test_gpu_agent.py tests/test_gpu_configs.py -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/r03_c/agent_tests.log 2>&1 || { echo AGENT TESTS FAILED; tail -40 gpurun_out/r03_c/agent_tests.log; exit 1; }
tail -2 gpurun_out/r03_c/agent_tests.log
bash tools/gpu_session.sh r03_c ubench bdq
