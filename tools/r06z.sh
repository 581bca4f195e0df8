cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/r06_z; mkdir -p $out; export TMPDIR=/tmp
export PBN_SETTLE_SPLIT=0
for n in 32768 65536; do
  timeout -k 10 120 python tools/stamps.py --settle 64 --rollout 20 --envs $n > $out/sstamps_$n.json 2> $out/sstamps_$n.err || { tail -5 $out/sstamps_$n.err; exit 3; }
done
echo done
