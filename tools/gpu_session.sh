#!/bin/bash
# One gpurun session on the GPU box, as a list of steps (replaces round 2's one-script-per-call
# tools/gpu_r02_*.sh).  Usage:
#   tools/gpu_session.sh TAG STEP [STEP ...]
# Outputs under gpurun_out/TAG/.  Every GPU step runs under its own time limit; the first
# failure ends the session (no retries).  Steps:
#   tests            the -m gpu suite (tools/gpu_tests.sh) + smoke()
#   pytest:F1,F2     the -m gpu tests of those files only (e.g. pytest:tests/test_gpu_agent.py)
#   driver           the driver's bench command (--gpus 1 --steps 20 --warmup 5) + kernel trace + PMC
#   s2000            2,000 steps at 65,536 envs (100-step launches) + kernel trace + PMC
#   1m               pbn28 x 1,048,576 envs, 500 steps
#   8m               pbn28 x 8,388,608 envs, 200 steps
#   pbn70            config 3: pbn70 x 1,048,576 envs, 200 steps
#   bdq              config 5: the BDQ frame at 32,768 envs (+ kernel trace)
#   bdq-learn        BDQ training frames at 32,768 envs (+ kernel trace)
#   stamps           the pipelined kernel's per-role segment clocks at iteration 10 (diagnostic build
#                    pbn_rl_amd/libpbn_env_stamps.so: tools/stamps.py --build), 20- and 100-step launches
#   sstamps          the settle kernel's per-role segment clocks (stamps build; tools/stamps.py --settle 64)
#   qstamps          config 5's Q-network launch per-phase clocks (stamps build; tools/qnet_stamps.py)
#   lstamps          the fused learner update's per-phase clocks (stamps build; tools/learn_stamps.py)
#   settle           the driver's command (with its settle_law and hand-off fields) and config 2 under the
#                    settle law alone (--settle 64, 200 steps) + its kernel trace
#   bdqpmc           the BDQ frame under two PMC passes: L2 hits / misses / requests, HBM fetch + write
#   handoff          the world-1 hand-off pass alone (tools/handoff_trace.py, plans 20 and 10,10) and its
#                    rocprofv3 kernel + memory-copy trace, attributed per rep
#   handoff100       the world-1 hand-off pass of four 100-step launches (the 2,000-step line's plan) and its
#                    kernel + memory-copy trace
#   budget           the one-update kernel's instruction and LDS counters at 2,000 steps (65,536 envs)
#                    and at 1M envs, two PMC passes each, for tools/isa_budget.py --pmc (issue model)
#   ubench           tools/ubench_valu_issue (VALU issue rates by instruction and waves per SIMD)
#   nofinal          the driver's command and 2,000 steps without s' (--no-final-state)
#   abenv            every pbn_rl_amd/libpbn_env_diag_*.so but diag_s_*, then this tree: tests/test_gpu_parity.py,
#                    the driver's command, 2,000 steps and 1M envs (env rollout variants)
#   abbdq            every pbn_rl_amd/libpbn_env_diag_q*.so, then this tree: tests/test_gpu_agent.py
#                    and the BDQ frame (frame and tail-launch times; Q-network tail variants)
#   ab70             A/B: pbn70 x 1M and pbn28 x 1M, pbn_rl_amd/libpbn_env_diag_base.so, then this tree
#   abgather         every pbn_rl_amd/libpbn_env_diag_g_*.so, then this tree: the driver's command and 2,000
#                    steps with the hand-off passes (value_with_gather; hand-off variants)
#   ablearn          every pbn_rl_amd/libpbn_env_diag_l_*.so, then this tree: tests/test_gpu_learn.py and
#                    the BDQ training frame (learner kernel variants)
#   absettle         every pbn_rl_amd/libpbn_env_diag_s_*.so, then this tree: tests/test_gpu_settle.py,
#                    the settle law at the driver's shape (20 steps) and at 200 steps (settle kernel variants)
#   ab               A/B: the driver's command, 2,000 steps and the BDQ frame, first with
#                    pbn_rl_amd/libpbn_env_diag_base.so (tools/ab_build.sh REV), then this tree
set -o pipefail
shopt -s nullglob   # a variant glob with no match expands to nothing
tag=$1; shift
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
fail() { echo "STEP $1 FAILED"; exit 1; }
bench() {   # bench NAME ARGS... : one bench line
  local name=$1; shift
  timeout -k 10 300 python bench.py "$@" > "$out/$name.json" 2> "$out/$name.err" || fail "$name"
  echo "$name: $(python -c "import json; d=[json.loads(l) for l in open('$out/$name.json') if l.startswith('{')][-1]; print(d['value'], d.get('roofline',{}).get('frac'))")"
}
for step in "$@"; do
  case $step in
    tests) bash tools/gpu_tests.sh "$tag/tests" || fail tests ;;
    pytest:*)
      files=${step#pytest:}
      timeout -k 10 ${PYTEST_TIMEOUT:-600} python -u -m pytest ${files//,/ } -m gpu -x -v --timeout 240 --timeout-method thread \
        > "$out/pytest.log" 2>&1 || { tail -40 "$out/pytest.log"; fail "$step"; }
      tail -2 "$out/pytest.log" ;;
    driver) bash tools/gpu_bench_profile.sh "$tag/driver" --gpus 1 --steps 20 --warmup 5 || fail driver ;;
    s2000) bash tools/gpu_bench_profile.sh "$tag/s2000" --gpus 1 --steps 2000 --warmup 200 || fail s2000 ;;
    1m) bench bench_1m --envs 1048576 --steps 500 --warmup 100 --no-cpu-baseline ;;
    8m) bench bench_8m --envs 8388608 --steps 200 --warmup 20 --no-cpu-baseline --no-gather ;;
    pbn70) bench bench_pbn70 --network pbn70 --envs 1048576 --steps 200 --warmup 20 ;;
    bdq)
      bench bench_bdq --workload bdq
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/bdq_trace" -o run -- \
        python bench.py --workload bdq --no-cpu-baseline > "$out/bdq_trace.json" 2> "$out/bdq_trace.err" || fail bdq-trace ;;
    bdqpmc)
      timeout -k 10 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum --kernel-trace --stats --output-format csv \
        -d "$out/bdq_pmc_l2" -o run -- python bench.py --workload bdq --no-cpu-baseline > /dev/null 2> "$out/bdq_pmc_l2.err" || fail bdqpmc-l2
      timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --stats --output-format csv \
        -d "$out/bdq_pmc_fetch" -o run -- python bench.py --workload bdq --no-cpu-baseline > /dev/null 2> "$out/bdq_pmc_fetch.err" || fail bdqpmc-fetch
      timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --stats --output-format csv \
        -d "$out/bdq_pmc_write" -o run -- python bench.py --workload bdq --no-cpu-baseline > /dev/null 2> "$out/bdq_pmc_write.err" || fail bdqpmc-write
      echo "bdqpmc done" ;;
    bdq-learn)
      bench bench_bdq_learn --workload bdq-learn
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/bdq_learn_trace" -o run -- \
        python bench.py --workload bdq-learn > "$out/bdq_learn_trace.json" 2> "$out/bdq_learn_trace.err" || fail bdq-learn-trace
      # (every dispatch's row: tens of MB; the stats stay)
      find "$out/bdq_learn_trace" -name '*kernel_trace.csv' -delete ;;
    stamps)
      for T in 20 100; do
        timeout -k 10 120 python tools/stamps.py --pipe --rollout $T > "$out/stamps_T$T.json" 2> "$out/stamps_T$T.err" \
          || fail "stamps T$T"
      done
      echo "stamps done" ;;
    sstamps)
      for T in 20 100; do
        timeout -k 10 120 python tools/stamps.py --settle 64 --rollout $T > "$out/settle_stamps_T$T.json" \
          2> "$out/settle_stamps_T$T.err" || fail "sstamps T$T"
      done
      echo "sstamps done" ;;
    qstamps)
      timeout -k 10 180 python tools/qnet_stamps.py > "$out/qstamps.json" 2> "$out/qstamps.err" || fail qstamps
      echo "qstamps done" ;;
    lstamps)
      timeout -k 10 180 python tools/learn_stamps.py > "$out/learn_stamps.json" 2> "$out/learn_stamps.err" \
        || fail lstamps
      echo "lstamps done" ;;
    settle)
      bench bench_driver --gpus 1 --steps 20 --warmup 5
      bench bench_settle64 --settle 64 --steps 200 --warmup 20 --no-cpu-baseline --no-gather
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/settle_trace" -o run -- \
        python bench.py --settle 64 --steps 200 --warmup 20 --no-cpu-baseline --no-gather \
        > "$out/settle_trace.json" 2> "$out/settle_trace.err" || fail settle-trace ;;
    handoff)
      for plan in 20 10,10; do
        timeout -k 10 180 python tools/handoff_trace.py --plan $plan > "$out/handoff_${plan/,/_}.json" 2> "$out/handoff.err" \
          || fail "handoff $plan"
        cat "$out/handoff_${plan/,/_}.json"
      done
      timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d "$out/handoff_trace" -o run -- \
        python tools/handoff_trace.py --plan 20 > "$out/handoff_trace.json" 2> "$out/handoff_trace.err" || fail handoff-trace
      python tools/handoff_trace.py --summarize "$out/handoff_trace" > "$out/handoff_summary.json" || fail handoff-summary
      echo "handoff done" ;;
    handoff100)
      timeout -k 10 180 python tools/handoff_trace.py --plan 100,100,100,100 --reps 10 > "$out/handoff_100x4.json" \
        2> "$out/handoff100.err" || fail "handoff100"
      cat "$out/handoff_100x4.json"
      timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d "$out/handoff100_trace" -o run -- \
        python tools/handoff_trace.py --plan 100,100,100,100 --reps 10 > "$out/handoff100_trace.json" \
        2> "$out/handoff100_trace.err" || fail handoff100-trace
      python tools/handoff_trace.py --summarize "$out/handoff100_trace" > "$out/handoff100_summary.json" || fail handoff100-summary
      echo "handoff100 done" ;;
    budget)
      for shape in "s2000:--steps 2000 --warmup 200" "1m:--envs 1048576 --steps 500 --warmup 100"; do
        nm=${shape%%:*}; args=${shape#*:}
        timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_WR \
          SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --kernel-trace --stats --output-format csv \
          -d "$out/budget_${nm}_a" -o run -- python bench.py --no-cpu-baseline --no-gather --settle-line 0 $args \
          > "$out/budget_${nm}_a.json" 2> "$out/budget_${nm}_a.err" || fail "budget-$nm-a"
        timeout -k 10 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS \
          SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE --kernel-trace --stats \
          --output-format csv -d "$out/budget_${nm}_b" -o run -- python bench.py --no-cpu-baseline --no-gather \
          --settle-line 0 $args > "$out/budget_${nm}_b.json" 2> "$out/budget_${nm}_b.err" || fail "budget-$nm-b"
        echo "budget $nm done"
      done ;;
    ubench)
      timeout -k 10 300 tools/ubench_valu_issue > "$out/ubench_valu_issue.jsonl" 2> "$out/ubench.err" || fail ubench
      echo "ubench done" ;;
    nofinal)
      bench bench_driver_nofinal --gpus 1 --steps 20 --warmup 5 --no-final-state --no-cpu-baseline
      bench bench_s2000_nofinal --steps 2000 --warmup 200 --no-final-state --no-cpu-baseline ;;
    abbdq)
      for lib in pbn_rl_amd/libpbn_env_diag_q*.so tree; do
        side=$(basename "$lib" .so); side=${side#libpbn_env_diag_}
        if [ "$lib" = tree ]; then unset PBN_LIB; else export PBN_LIB=$PWD/$lib; fi
        timeout -k 10 300 python -u -m pytest tests/test_gpu_agent.py -m gpu -x -q --timeout 120 --timeout-method thread \
          > "$out/abbdq_${side}_agent.log" 2>&1 || { tail -20 "$out/abbdq_${side}_agent.log"; fail "abbdq $side agent"; }
        timeout -k 10 300 python bench.py --workload bdq --no-cpu-baseline > "$out/abbdq_$side.json" 2> "$out/abbdq_$side.err" \
          || fail "abbdq $side"
        python -c "import json; d=[json.loads(l) for l in open('$out/abbdq_$side.json') if l.startswith('{')][-1]; r=d['roofline']; print('$side frame_ms', d['ms_per_step'], 'tail_ms', r['launch_ms'], 'bilinear_ms', r.get('bilinear', {}).get('launch_ms'))"
      done
      unset PBN_LIB ;;
    ab)
      for side in base tree; do
        if [ $side = base ]; then export PBN_LIB=$PWD/pbn_rl_amd/libpbn_env_diag_base.so; else unset PBN_LIB; fi
        bench ab_${side}_driver --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-gather
        bench ab_${side}_s2000 --steps 2000 --warmup 200 --no-cpu-baseline --no-gather
        bench ab_${side}_bdq --workload bdq --no-cpu-baseline
      done
      unset PBN_LIB ;;
    ab70)
      for side in base tree; do
        if [ $side = base ]; then export PBN_LIB=$PWD/pbn_rl_amd/libpbn_env_diag_base.so; else unset PBN_LIB; fi
        bench ab70_${side}_pbn70 --network pbn70 --envs 1048576 --steps 200 --warmup 20 --no-cpu-baseline --no-gather
        bench ab70_${side}_1m --envs 1048576 --steps 300 --warmup 50 --no-cpu-baseline --no-gather
      done
      unset PBN_LIB ;;
    abenv)
      for lib in pbn_rl_amd/libpbn_env_diag_[!s]*.so tree; do
        side=$(basename "$lib" .so); side=${side#libpbn_env_diag_}
        if [ "$lib" = tree ]; then unset PBN_LIB; else export PBN_LIB=$PWD/$lib; fi
        timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
          > "$out/abenv_${side}_parity.log" 2>&1 || { tail -20 "$out/abenv_${side}_parity.log"; fail "abenv $side parity"; }
        bench abenv_${side}_driver --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-gather --settle-line 0
        bench abenv_${side}_s2000 --steps 2000 --warmup 200 --no-cpu-baseline --no-gather --settle-line 0
        bench abenv_${side}_1m --envs 1048576 --steps 300 --warmup 50 --no-cpu-baseline --no-gather --settle-line 0
      done
      unset PBN_LIB ;;
    abgather)
      for lib in pbn_rl_amd/libpbn_env_diag_g_*.so tree; do
        side=$(basename "$lib" .so); side=${side#libpbn_env_diag_g_}
        if [ "$lib" = tree ]; then unset PBN_LIB; else export PBN_LIB=$PWD/$lib; fi
        bench abgather_${side}_driver --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --settle-line 0
        bench abgather_${side}_s2000 --steps 2000 --warmup 200 --no-cpu-baseline --settle-line 0
        python -c "import json; d=[json.loads(l) for l in open('$out/abgather_${side}_s2000.json') if l.startswith('{')][-1]; print('  with_gather / value', d['value_with_gather'] / d['value'])"
      done
      unset PBN_LIB ;;
    ablearn)
      for lib in pbn_rl_amd/libpbn_env_diag_l_*.so tree; do
        side=$(basename "$lib" .so); side=${side#libpbn_env_diag_l_}
        if [ "$lib" = tree ]; then unset PBN_LIB; else export PBN_LIB=$PWD/$lib; fi
        timeout -k 10 300 python -u -m pytest tests/test_gpu_learn.py -m gpu -x -q --timeout 120 --timeout-method thread \
          > "$out/ablearn_${side}_learn.log" 2>&1 || { tail -20 "$out/ablearn_${side}_learn.log"; fail "ablearn $side"; }
        bench ablearn_${side}_frame --workload bdq-learn --no-cpu-baseline
      done
      unset PBN_LIB ;;
    absettle)
      for lib in pbn_rl_amd/libpbn_env_diag_s_*.so tree; do
        side=$(basename "$lib" .so); side=${side#libpbn_env_diag_s_}
        if [ "$lib" = tree ]; then unset PBN_LIB; else export PBN_LIB=$PWD/$lib; fi
        timeout -k 10 300 python -u -m pytest tests/test_gpu_settle.py -m gpu -x -q --timeout 120 --timeout-method thread \
          > "$out/absettle_${side}_settle.log" 2>&1 || { tail -20 "$out/absettle_${side}_settle.log"; fail "absettle $side"; }
        bench absettle_${side}_d20 --gpus 1 --steps 20 --warmup 5 --settle 64 --no-cpu-baseline --no-gather
        bench absettle_${side}_s200 --steps 200 --warmup 20 --settle 64 --no-cpu-baseline --no-gather
        timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --stats --output-format csv \
          -d "$out/absettle_${side}_write" -o run -- python bench.py --steps 20 --warmup 5 --settle 64 \
          --no-cpu-baseline --no-gather > /dev/null 2> "$out/absettle_${side}_write.err" || fail "absettle $side write"
      done
      unset PBN_LIB ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "SESSION $tag DONE"
