cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/r06_r; mkdir -p $out; export TMPDIR=/tmp
for side in tree rc16 tree rc16; do
  if [ $side = tree ]; then unset PBN_LIB; else export PBN_LIB=$PWD/pbn_rl_amd/libpbn_env_diag_l_$side.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/$side$RANDOM -o run -- \
    python bench.py --workload bdq-learn --no-cpu-baseline > $out/$side.json 2> $out/$side.err || { tail -5 $out/$side.err; exit 3; }
  find $out/$side -name '*kernel_trace.csv' -delete
  python -c "import json; d=[json.loads(l) for l in open('$out/$side.json') if l.startswith('{')][-1]; print('$side', d['ms_per_step'], d['roofline'].get('update',{}).get('update_ms'))"
  f=$(find $out/$side -name '*kernel_stats.csv'); grep -E "learn_(fwd|bwd|apply)" $f | cut -d, -f1-4
done
