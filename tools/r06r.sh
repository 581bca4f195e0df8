# A/B of learner variants (pbn_rl_amd/libpbn_env_diag_l_<name>.so) against this tree:
#   bash tools/r06r.sh TAG NAME [NAME ...]   (two alternating rounds; bdq-learn under the kernel trace)
cd "$GRAFT_REPO_ROOT" || exit 1
tag=$1; shift
out=gpurun_out/$tag; mkdir -p $out; export TMPDIR=/tmp
for rep in 1 2; do
for side in tree "$@"; do
  if [ $side = tree ]; then unset PBN_LIB; else export PBN_LIB=$PWD/pbn_rl_amd/libpbn_env_diag_l_$side.so; fi
  d=$out/${side}_$rep
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- \
    python bench.py --workload bdq-learn --no-cpu-baseline > $d.json 2> $d.err || { tail -5 $d.err; exit 3; }
  find $d -name '*kernel_trace.csv' -delete
  python -c "import json; d=[json.loads(l) for l in open('$d.json') if l.startswith('{')][-1]; print('$side', d['value'], d['ms_per_step'], d['roofline'].get('update',{}).get('update_ms'))"
  f=$(find $d -name '*kernel_stats.csv'); grep -E "learn_(fwd|bwd|apply)" $f | cut -d, -f1-4
done
done
