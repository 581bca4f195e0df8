# A/B of the one-step wave kernel's prologue (diagnostic library diag_q_step) on the BDQ frames
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/r06_ah; mkdir -p $out; export TMPDIR=/tmp
PBN_LIB=$PWD/pbn_rl_amd/libpbn_env_diag_q_step.so timeout -k 10 900 python -u -m pytest tests/test_gpu_agent.py tests/test_gpu_graph.py tests/test_gpu_configs.py -m gpu -x -q --timeout 240 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 4; }
tail -1 $out/tests.log
for rep in 1 2; do
for side in tree step; do
  if [ $side = tree ]; then unset PBN_LIB; else export PBN_LIB=$PWD/pbn_rl_amd/libpbn_env_diag_q_$side.so; fi
  d=$out/${side}_$rep
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- \
    python bench.py --workload bdq --no-cpu-baseline > $d.json 2> $d.err || { tail -5 $d.err; exit 3; }
  find $d -name '*kernel_trace.csv' -delete
  python -c "import json; d=[json.loads(l) for l in open('$d.json') if l.startswith('{')][-1]; print('$side', d['value'], d['ms_per_step'])"
  python -c "
import csv,glob
for r in csv.DictReader(open(glob.glob('$d/*kernel_stats.csv')[0])):
    if 'step_wave' in r['Name'] or 'qnet_tail' in r['Name']: print('  ', r['Name'][:50], round(float(r['AverageNs'])/1000,2))"
  timeout -k 10 300 python bench.py --workload bdq-learn --no-cpu-baseline > ${d}_learn.json 2> ${d}_learn.err || { tail -5 ${d}_learn.err; exit 3; }
  python -c "import json; d=[json.loads(l) for l in open('${d}_learn.json') if l.startswith('{')][-1]; print('$side learn', d['value'], d['ms_per_step'])"
done
done
unset PBN_LIB
