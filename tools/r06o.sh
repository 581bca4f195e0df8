cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/r06_t; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_replay.py tests/test_gpu_graph.py tests/test_gpu_learn.py tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_agent.py -m gpu -x -q --timeout 240 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 4; }
tail -1 $out/tests.log
for rep in 1 2; do
for side in base tree; do
  if [ $side = base ]; then cd ab_base_tree; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$out/${side}_$rep -o run -- \
    python bench.py --workload bdq-learn --no-cpu-baseline > $GRAFT_REPO_ROOT/$out/${side}_$rep.json 2> $GRAFT_REPO_ROOT/$out/${side}_$rep.err || { tail -5 $GRAFT_REPO_ROOT/$out/${side}_$rep.err; exit 3; }
  cd "$GRAFT_REPO_ROOT"
  find $out/${side}_$rep -name '*kernel_trace.csv' -delete
  python -c "import json; d=[json.loads(l) for l in open('$out/${side}_$rep.json') if l.startswith('{')][-1]; print('$side', d['value'], d['ms_per_step'], d['roofline'].get('update',{}).get('update_ms'))"
  f=$(find $out/${side}_$rep -name '*kernel_stats.csv'); grep -E "learn_(fwd|bwd|apply)|pack" $f | cut -d, -f1-4
done
done
