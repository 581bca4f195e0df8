"""Operator-level profile of the BDQ training frame (bench.py --workload bdq-learn's learner, eager).

  python tools/learn_profile.py [--envs 32768] [--frames 20]

torch.profiler over eager frames after warm-up: per PyTorch operator its calls per frame and device
time per frame, so the PyTorch update's ~170 kernels can be attributed to its operations.  Profiles
the PyTorch update (fused=False); the default learner's fused update is three HIP launches
(tools/learn_stamps.py times their phases).
"""
import argparse
import json
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=32768)
    ap.add_argument("--frames", type=int, default=20)
    args = ap.parse_args()
    import torch
    from torch.profiler import ProfilerActivity, profile

    from pbn_rl_amd.agent import BranchingQNetwork
    from pbn_rl_amd.attractors import load_attractors
    from pbn_rl_amd.network import load_network
    from pbn_rl_amd.replay import BDQLearner
    from pbn_rl_amd.spec import EnvSpec
    from pbn_rl_amd.vector_env import VectorPBNEnv

    dev = torch.device("cuda", 0)
    if os.environ.get("PBN_BLAS"):   # "cublas" = rocBLAS on ROCm, "cublaslt" = hipBLASLt (torch's default)
        torch.backends.cuda.preferred_blas_library(os.environ["PBN_BLAS"])
    spec = EnvSpec(load_network("pbn28"), load_attractors("pbn28"), perturbation=0.01, prob_bits=16, horizon=20)
    env = VectorPBNEnv(spec, args.envs, seed=0, device=dev, keep_final_state=True)
    env.reset()
    torch.manual_seed(0)
    learner = BDQLearner(env, BranchingQNetwork((spec.n, spec.n), spec.n + 1, 3), capacity=4 * args.envs,
                         learning_starts=256, epsilon_start=0.0, epsilon_final=0.0, fused=False)
    for _ in range(10):
        learner.frame()
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
        for _ in range(args.frames):
            learner.frame()
        torch.cuda.synchronize()
    rows = []
    for e in prof.key_averages():
        dev_us = getattr(e, "self_device_time_total", None)
        if dev_us is None:
            dev_us = getattr(e, "self_cuda_time_total", 0)
        if dev_us <= 0:
            continue
        rows.append({"op": e.key, "calls_per_frame": e.count / args.frames,
                     "device_us_per_frame": dev_us / args.frames})
    rows.sort(key=lambda r: -r["device_us_per_frame"])
    gemms = []   # the matrix products by operand shapes
    for e in prof.key_averages(group_by_input_shape=True):
        if e.key not in ("aten::mm", "aten::addmm", "aten::bmm", "aten::baddbmm"):
            continue
        dev_us = getattr(e, "device_time_total", None) or getattr(e, "cuda_time_total", 0)
        gemms.append({"op": e.key, "shapes": str(e.input_shapes), "calls_per_frame": e.count / args.frames,
                      "device_us_per_frame": dev_us / args.frames})
    gemms.sort(key=lambda r: -r["device_us_per_frame"])
    print(json.dumps({"frames": args.frames, "envs": args.envs, "blas": str(torch.backends.cuda.preferred_blas_library()),
                      "device_us_per_frame": sum(r["device_us_per_frame"] for r in rows), "ops": rows[:60],
                      "gemms": gemms},
                     indent=1))


if __name__ == "__main__":
    main()
