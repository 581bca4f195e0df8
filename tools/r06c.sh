cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/r06_d; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_settle.py tests/test_gpu_configs.py tests/test_gpu_graph.py tests/test_gpu_replay.py tests/test_gpu_parity.py -m gpu -x -q --timeout 180 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 4; }
tail -2 $out/tests.log
timeout -k 10 120 python tools/facade_probe.py --network pbn28 > $out/facade28.json 2> $out/facade28.err || { tail $out/facade28.err; exit 5; }
cat $out/facade28.json
timeout -k 10 300 python bench.py --workload bdq --settle 64 > $out/bdq_settle.json 2> $out/bdq_settle.err || { tail $out/bdq_settle.err; exit 6; }
python -c "import json; d=[json.loads(l) for l in open('$out/bdq_settle.json') if l.startswith('{')][-1]; print('bdq settle64', d['value'], d['ms_per_step'])"
PBN_ROLL=lean timeout -k 10 300 python bench.py --workload bdq --settle 64 --no-cpu-baseline > $out/bdq_settle_lean.json 2> $out/bdq_settle_lean.err || { tail $out/bdq_settle_lean.err; exit 6; }
python -c "import json; d=[json.loads(l) for l in open('$out/bdq_settle_lean.json') if l.startswith('{')][-1]; print('bdq settle64 lean', d['value'], d['ms_per_step'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/bdq_settle_trace -o run -- python bench.py --workload bdq --settle 64 --no-cpu-baseline > $out/bdq_settle_trace.json 2> $out/bdq_settle_trace.err || { tail $out/bdq_settle_trace.err; exit 7; }
