# the settle kernel's split selection: tests, then the BDQ settle frame and the settle lines with
# PBN_SETTLE_SPLIT forced 0 / 1 (same library), two alternating rounds
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/r06_y; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_settle.py tests/test_gpu_configs.py tests/test_gpu_replay.py tests/test_gpu_graph.py -m gpu -x -q --timeout 240 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 4; }
tail -1 $out/tests.log
line() { python -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; print(sys.argv[2], d['value'], d['ms_per_step'])" "$@"; }
for rep in 1 2; do
for sp in 0 1; do
  export PBN_SETTLE_SPLIT=$sp
  timeout -k 10 300 python bench.py --workload bdq --settle 64 --no-cpu-baseline > $out/bdq_s${sp}_$rep.json 2> $out/bdq_s${sp}_$rep.err || { tail -5 $out/bdq_s${sp}_$rep.err; exit 3; }
  line $out/bdq_s${sp}_$rep.json "bdq_settle64 split=$sp"
  timeout -k 10 300 python bench.py --settle 64 --steps 20 --warmup 5 --no-cpu-baseline --no-gather --settle-line 0 > $out/d20_s${sp}_$rep.json 2> $out/d20_s${sp}_$rep.err || { tail -5 $out/d20_s${sp}_$rep.err; exit 3; }
  line $out/d20_s${sp}_$rep.json "settle64_T20 split=$sp"
  timeout -k 10 300 python bench.py --settle 64 --steps 200 --warmup 20 --no-cpu-baseline --no-gather --settle-line 0 > $out/s200_s${sp}_$rep.json 2> $out/s200_s${sp}_$rep.err || { tail -5 $out/s200_s${sp}_$rep.err; exit 3; }
  line $out/s200_s${sp}_$rep.json "settle64_T200 split=$sp"
done
done
unset PBN_SETTLE_SPLIT
