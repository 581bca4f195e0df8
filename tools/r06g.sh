cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu_session.sh r06_g tests driver s2000 settle 1m pbn70 bdq || exit 1
bash tools/gpu_bench_profile.sh r06_g/settle100 --steps 200 --warmup 20 --settle 64 --no-cpu-baseline --no-gather || exit 2
bash tools/gpu_bench_profile.sh r06_g/settle20 --steps 20 --warmup 5 --settle 64 --no-cpu-baseline --no-gather || exit 3
echo ALL DONE
