"""bench.py's host-side arithmetic (no GPU): the algorithmic byte and FLOP counts the
roofline is computed from (DESIGN.md "Kernels"), the launch plan, and the parameter count
of the Q-network the FLOP formula describes."""
import sys

import pytest

import bench
from pbn_rl_amd.agent import BranchingQNetwork


def test_rollout_bytes_match_design():
    # 12 + 13 T bytes per env per launch for one state word; 1,312 B at T = 100
    assert bench.rollout_bytes_per_env(1, 100) == 1312
    assert bench.rollout_bytes_per_env(1, 100) * 65536 == 85983232        # profiles/pmc_*: algorithmic
    assert bench.rollout_bytes_per_env(3, 1) == 2 * (12 + 2) + 12 + 12 + 5


def test_step_bytes():
    assert bench.algorithmic_bytes_per_env(1) == 20                        # 20 B/env-step
    assert bench.algorithmic_bytes_per_env(2) == 32


def test_survey_bytes_price_the_roofline():
    # 20 B/env-step up to 32 nodes (u32 state), 56 B for pbn70 (2 x u64 state)
    assert bench.survey_bytes_per_env_step(7) == bench.survey_bytes_per_env_step(28) == 20
    assert bench.survey_bytes_per_env_step(32) == 20
    assert bench.survey_bytes_per_env_step(70) == bench.survey_bytes_per_env_step(128) == 56
    assert bench.survey_bytes_per_env_step(33) == 3 * 8 + 8


@pytest.mark.parametrize("steps,chunk", [(2000, 100), (250, 100), (7, 3), (5, 10), (0, 4)])
def test_launch_plan(steps, chunk):
    plan = bench.launch_plan(steps, chunk)
    assert sum(plan) == steps and all(0 < k <= chunk for k in plan)
    assert all(k == chunk for k in plan[:-1])


@pytest.mark.parametrize("n", [7, 28, 70])
def test_qnet_flops_count_every_weight(n):
    """2 x (multiply-adds) = 2 x (weights), since every weight is used once per env."""
    net = BranchingQNetwork((n, n), n + 1, 3)
    weights = sum(p.numel() for name, p in net.named_parameters() if name.endswith("weight"))
    assert bench.qnet_flops_per_env(n) == 2 * weights


def test_parse_defaults(monkeypatch):
    monkeypatch.setattr(sys, "argv", ["bench.py"])
    a = bench.parse()
    assert (a.gpus, a.steps, a.warmup, a.envs, a.network, a.chunk) == (1, 2000, 200, 65536, "pbn28", 100)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--workload", "bdq"])
    a = bench.parse()
    assert (a.steps, a.warmup, a.envs) == (200, 20, 32768)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--workload", "bdq-learn"])
    a = bench.parse()
    assert a.learn_graph and a.no_graph and not a.no_cpu_baseline   # the training frame's own CPU baseline


def test_multi_gpu_request_without_gpus_fails_loudly():
    """`bench.py --gpus 2` launches its own ranks; with fewer GPUs than ranks it must refuse
    (exit 2) instead of rehearsing several ranks on one device."""
    import os
    import subprocess

    r = subprocess.run([sys.executable, bench.__file__, "--gpus", "2", "--steps", "1"], capture_output=True,
                       text=True, timeout=300, env=dict(os.environ, HIP_VISIBLE_DEVICES=""))
    assert r.returncode == 2 and "--gpus 2" in r.stderr
    r = subprocess.run([sys.executable, bench.__file__, "--gpus", "1"], capture_output=True, text=True,
                       timeout=300, env=dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0"))
    assert r.returncode == 2 and "WORLD_SIZE=2" in r.stderr


def test_usable_cpus():
    info = bench.usable_cpus()
    assert 1 <= info["usable"] <= info["affinity"] <= info["cpu_count"]
    if info["cgroup_quota"] is not None:
        assert info["usable"] <= max(1, -(-info["cgroup_quota"] // 1))


def test_visible_gpu_count_does_not_initialise_hip(tmp_path, monkeypatch):
    """The parent of `bench.py --gpus N` counts GPUs from sysfs and the visibility variables,
    never through HIP (torch.cuda stays uninitialised), and honours the variables."""
    import torch
    n = bench.visible_gpu_count()
    assert n >= 0 and not torch.cuda.is_initialized()
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "")
    assert bench.visible_gpu_count() == 0
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "0")
    assert bench.visible_gpu_count() <= 1


def test_spawn_path_in_a_fresh_interpreter_never_touches_hip():
    """Run the parent's pre-spawn code in a clean interpreter: after counting, torch.cuda is not
    initialised (the ranks get the device)."""
    import subprocess
    code = ("import sys; sys.argv=['bench.py']; import bench, torch; bench.visible_gpu_count(); "
            "print(torch.cuda.is_initialized())")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300,
                       cwd=str(__import__('pathlib').Path(bench.__file__).parent))
    assert r.returncode == 0 and r.stdout.strip().endswith("False"), r.stderr


def test_qnet_tail_flops_count_the_layers_after_the_bilinear():
    import bench
    # Bittner-28, 3 branches: trunk 256*128 + 128*64 + 64*32, 4 first head layers 32*64,
    # value 64*1, 3 advantage layers 64*29 multiply-adds
    macs = 32768 + 8192 + 2048 + 4 * 2048 + 64 + 3 * 64 * 29
    assert bench.qnet_tail_flops_per_env(28, 3) == 2 * macs
    assert bench.qnet_flops_per_env(28, 3) - bench.qnet_tail_flops_per_env(28, 3) == 2 * 28 * 28 * 256


def test_settle_stats_iterations_and_launch_tail():
    """pbn_rollout_settle's per-env plans: an env spends its updates plus one dropped speculation
    per step that settles before the cap; a launch lasts as long as its busiest env."""
    import torch
    u = torch.ones(3, 64, dtype=torch.int16)
    u[0, 5] = 40          # step 0, env 5: 40 updates, below the cap
    u[2, 63] = 64         # step 2, env 63: capped (no dropped speculation)
    s = bench.settle_stats([u], 1.0, 192, cap=64)
    assert s["mean_updates_per_env_step"] == pytest.approx((192 - 2 + 40 + 64) / 192)
    per_env = [6.0] * 64
    per_env[5] = 41 + 2 + 2
    per_env[63] = 2 + 2 + 64
    assert s["mean_env_iterations_per_step"] == pytest.approx(sum(per_env) / 64 / 3)
    assert s["launch_iterations_per_step"] == pytest.approx(68 / 3)
    assert s["launch_tail"] == pytest.approx(68 / (sum(per_env) / 64))
    assert s["updates_quantiles"]["max"] == 64


def test_update_flops_are_five_row_forwards():
    assert bench.update_flops(28, 256) == 5 * 256 * bench.qnet_flops_per_env(28)
    assert bench.update_flops(7, 32, 2) == 5 * 32 * bench.qnet_flops_per_env(7, 2)


def test_cpu_training_frame_baseline_runs_one_update_per_frame():
    """bench.py --workload bdq-learn's cpu_baseline: acting frame + ring store + bdq_update on CPU."""
    import torch

    from pbn_rl_amd.attractors import load_attractors
    from pbn_rl_amd.network import load_network
    from pbn_rl_amd.spec import EnvSpec

    spec = EnvSpec(load_network("pbn7"), load_attractors("pbn7"), perturbation=0.01, horizon=20)
    torch.manual_seed(0)
    q = BranchingQNetwork((spec.n, spec.n), spec.n + 1, 3)
    before = [p.detach().clone() for p in q.parameters()]
    cb = bench.cpu_baseline_bdq_learn(spec, q, 256, 0.05, 1)
    assert cb["kind"] == "port" and cb["cores"] == 1 and cb["value"] > 0
    assert "update_policy" in cb["sample"]
    # the baseline trains a copy: the caller's network is untouched
    assert all(torch.equal(a, b) for a, b in zip(before, q.parameters()))
