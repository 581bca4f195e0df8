cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/r06_b; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_env.py tests/test_gpu_settle.py tests/test_gpu_law_pin.py tests/test_gpu_learn.py tests/test_gpu_rccl.py -m gpu -x -q --timeout 120 --timeout-method thread > $out/learn.log 2>&1 || { tail -30 $out/learn.log; exit 4; }
tail -2 $out/learn.log
timeout -k 10 120 python -c "
import bench, json
print(json.dumps(bench.config1_line('cuda:0', seconds=3.0)))" > $out/config1.json 2>$out/config1.err || { tail $out/config1.err; exit 5; }
cat $out/config1.json
for m in 1 2; do
PBN_PLANES_MAP=$m timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "planes or baseline" > $out/parity_$m.log 2>&1; rc=$?
tail -2 $out/parity_$m.log
[ $rc -eq 0 ] || exit $rc
done
for rep in 1 2; do
for v in pipe planes:0 planes:1 planes:2; do
  for s in 20 2000; do
    w=5; [ $s = 2000 ] && w=200
    PBN_ROLL=${v%%:*} PBN_PLANES_MAP=${v#*:} timeout -k 10 200 python bench.py --steps $s --warmup $w --no-cpu-baseline --no-gather --settle-line 0 > $out/b_${v}_$s.json 2> $out/b_${v}_$s.err || exit 3
    python -c "import json; d=[json.loads(l) for l in open('$out/b_${v}_$s.json') if l.startswith('{')][-1]; print('$v', $s, d['value'], d['ms_per_step'], d['roofline']['frac'])"
  done
done
done
