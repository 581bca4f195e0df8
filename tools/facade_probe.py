"""Where a scalar PBNEnv.step's time goes (config 1, the gym facade).

  python tools/facade_probe.py [--seconds 2]     (GPU box)

Times, per call, on pbn7 with the facade's default settle law: the whole env.step (as bench.py's
config1 line, minus its action draws); the pbn_step launch + pbn_stream_sync alone on the facade's
host group; an empty launch floor (pbn_copy_async of 16 bytes + pbn_stream_sync); the Python side
of env.step with the launch and sync replaced by no-ops.  Prints one JSON line."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def per_call(fn, seconds):
    for _ in range(50):
        fn()
    k, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        fn()
        k += 1
    return (time.perf_counter() - t0) / k * 1e6


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=2.0)
    ap.add_argument("--network", default="pbn7")
    args = ap.parse_args()
    import numpy as np
    import torch

    from pbn_rl_amd import _lib
    from pbn_rl_amd.env import PBNEnv
    env = PBNEnv(network=args.network, seed=7, device="cuda:0")
    env.reset()
    env.step([1])
    L = _lib.load()
    venv, hg = env._venv, env._hg
    stream = venv._stream()
    acts = [[1, 3], [], [2], [4, 5, 6]]
    i = [0]

    def step():
        _, _, term, trunc, _ = env.step(acts[i[0] & 3])
        i[0] += 1
        if term or trunc:
            env.reset()

    def launch_sync():
        nxt = 1 - hg.cur
        L.pbn_step(venv.net.handle, venv.seed, venv.step_index, venv.env_offset, venv.n_alloc, 0,
                   hg.dev[f"state{hg.cur}"], hg.dev["flip"], hg.dev["target"], hg.dev["t"], hg.dev[f"state{nxt}"], None,
                   hg.dev["reward"], hg.dev["flags"], stream)
        L.pbn_stream_sync(stream)

    buf = torch.zeros(64, dtype=torch.uint8, device="cuda")

    def floor():
        L.pbn_copy_async(buf.data_ptr(), buf.data_ptr() + 32, 16, stream)
        L.pbn_stream_sync(stream)

    def stream_handle():
        venv._stream()

    res = {"network": args.network, "settle": env.spec.settle,
           "env_step_us": per_call(step, args.seconds),
           "launch_sync_us": per_call(launch_sync, args.seconds),
           "empty_launch_sync_us": per_call(floor, args.seconds),
           "current_stream_lookup_us": per_call(stream_handle, args.seconds)}
    env.close()
    env = PBNEnv(network=args.network, seed=7, device="cuda:0", settle=0)
    env.reset()
    env.step([1])
    res["env_step_one_update_law_us"] = per_call(step, args.seconds)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
