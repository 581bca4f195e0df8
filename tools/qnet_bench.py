"""Time BranchingQNetwork forward variants on the GPU (config 5's dominant cost).

  python tools/qnet_bench.py [--envs 32768]

  ref     nn.Bilinear (torch's bilinear kernel path, as bdq_model/network.py runs it)
  gemm    pbn_rl_amd.agent.MyBilinear: one addmm over the outer product (the default)
  --train B[,B..]: also forward + backward of the whole network at these batch sizes for both
          MyBilinear forms (outer / contract), to place MyBilinear.contract_rows
Prints one JSON line per variant: ms per forward and TFLOP/s.
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from bench import qnet_flops_per_env  # noqa: E402
from pbn_rl_amd.agent import BranchingQNetwork  # noqa: E402


def time_fn(fn, iters=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=32768)
    ap.add_argument("--n", type=int, default=28)
    ap.add_argument("--train", default="")
    args = ap.parse_args()
    torch.manual_seed(0)
    net = BranchingQNetwork((args.n, args.n), args.n + 1, 3).cuda().eval()
    x = torch.randint(0, 2, (2, args.envs, args.n), device="cuda").float()
    bil = net.model[0].bilinear
    flops = args.envs * qnet_flops_per_env(args.n)
    with torch.no_grad():
        ref_first = lambda: bil(x[0], x[1])  # noqa: E731
        gemm_first = lambda: net.model[0](x)  # noqa: E731
        for name, fn in [("bilinear_ref", ref_first), ("bilinear_gemm", gemm_first), ("qnet_forward", lambda: net(x))]:
            ms = time_fn(fn)
            f = flops if name == "qnet_forward" else args.envs * 2 * args.n * args.n * 256
            print(json.dumps({"variant": name, "envs": args.envs, "ms": ms, "tflops": f / ms / 1e9}), flush=True)
        err = (ref_first() - gemm_first()).abs().max().item()
        print(json.dumps({"bilinear_max_abs_diff": err}))
    net.train()
    for B in [int(v) for v in args.train.split(",") if v]:
        xb = torch.randint(0, 2, (2, B, args.n), device="cuda").float()
        outs = {}
        for form in ("outer", "contract"):
            net.model[0].form = form

            def fb():
                net.zero_grad(set_to_none=True)
                q = net(xb)
                q.square().mean().backward()
                return q
            ms = time_fn(fb)
            with torch.no_grad():
                outs[form] = net(xb)
            print(json.dumps({"variant": f"fwd_bwd_{form}", "batch": B, "ms": ms}), flush=True)
        print(json.dumps({"batch": B, "forms_max_abs_diff": (outs["outer"] - outs["contract"]).abs().max().item()}))
        net.model[0].form = "auto"


if __name__ == "__main__":
    main()
