cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/r06_i; mkdir -p $out; export TMPDIR=/tmp
for pp in 2 1; do
PBN_PIPE_PAIRS=$pp timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_rccl.py tests/test_gpu_configs.py -m gpu -x -q --timeout 180 --timeout-method thread -k "not lean" > $out/tests_$pp.log 2>&1 || { tail -30 $out/tests_$pp.log; exit 4; }
tail -1 $out/tests_$pp.log
done
for rep in 1 2; do
for pp in 1 2; do
  for s in 20 2000; do
    w=5; [ $s = 2000 ] && w=200
    PBN_PIPE_PAIRS=$pp timeout -k 10 200 python bench.py --steps $s --warmup $w --no-cpu-baseline --no-gather --settle-line 0 > $out/b_${pp}_$s.json 2> $out/b_${pp}_$s.err || exit 3
    python -c "import json; d=[json.loads(l) for l in open('$out/b_${pp}_$s.json') if l.startswith('{')][-1]; print('pairs $pp', $s, d['value'], d['ms_per_step'])"
  done
done
PBN_PIPE_PAIRS=$pp timeout -k 10 200 python bench.py --envs 1048576 --steps 500 --warmup 100 --no-cpu-baseline --no-gather --settle-line 0 > $out/b1m_$rep.json 2>&1 || exit 5
python -c "import json; d=[json.loads(l) for l in open('$out/b1m_$rep.json') if l.startswith('{')][-1]; print('pairs 2 1m', d['value'])"
done
