cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/r06_an; mkdir -p $out; export TMPDIR=/tmp
PBN_LIB=$PWD/pbn_rl_amd/libpbn_env_diag_l_td4.so timeout -k 10 600 python -u -m pytest tests/test_gpu_learn.py tests/test_gpu_graph.py tests/test_gpu_replay.py -m gpu -x -q --timeout 240 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 4; }
tail -1 $out/tests.log
bash tools/r06r.sh r06_an td4
