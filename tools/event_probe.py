"""Timing-method probe: the driver's shape (one 20-step pbn_rollout at 65,536 envs) and a
one-element kernel, each between two HIP events behind the same spin gate as bench.py, with
torch's default events and with events created hipEventDisableSystemFence (no system-scope
release / acquire at the event, i.e. no write-back of device memory for the host).

    python tools/event_probe.py [--reps 30]   # one JSON line per method (medians, ms)
"""
import argparse
import ctypes
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

HIP_EVENT_DISABLE_SYSTEM_FENCE = 0x20000000


def hip_lib():
    return ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))


class NoFenceEvent:
    def __init__(self, hip):
        self.hip, self.ev = hip, ctypes.c_void_p()
        assert hip.hipEventCreateWithFlags(ctypes.byref(self.ev), HIP_EVENT_DISABLE_SYSTEM_FENCE) == 0

    def record(self, stream):
        assert self.hip.hipEventRecord(self.ev, ctypes.c_void_p(stream.cuda_stream)) == 0

    def elapsed_time(self, other):
        ms = ctypes.c_float()
        assert self.hip.hipEventSynchronize(other.ev) == 0
        assert self.hip.hipEventElapsedTime(ctypes.byref(ms), self.ev, other.ev) == 0
        return ms.value


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--steps", type=int, default=20)
    args = ap.parse_args()
    from pbn_rl_amd.attractors import load_attractors
    from pbn_rl_amd.network import load_network
    from pbn_rl_amd.spec import EnvSpec
    from pbn_rl_amd.vector_env import VectorPBNEnv

    dev = torch.device("cuda", 0)
    spec = EnvSpec(load_network("pbn28"), load_attractors("pbn28"), perturbation=0.01)
    env = VectorPBNEnv(spec, 65536, seed=0, device=dev)
    env.reset()
    stream = torch.cuda.Stream(device=dev)
    bufs = env.rollout_buffers(args.steps, keep_obs=True, keep_final=True)
    tiny = torch.zeros(1, device=dev)
    hip = hip_lib()

    def launch():
        env.rollout(args.steps, random_actions=True, keep_obs=True, keep_final=True, out=bufs)

    def timed(fn, make_event):
        torch.cuda.synchronize(dev)
        e0, e1 = make_event(), make_event()
        with torch.cuda.stream(stream):
            torch.cuda._sleep(250_000)
            e0.record(stream)
            fn()
            e1.record(stream)
        torch.cuda.synchronize(dev)
        return e0.elapsed_time(e1)

    makers = {"torch_default": lambda: torch.cuda.Event(enable_timing=True),
              "no_system_fence": lambda: NoFenceEvent(hip)}
    with torch.cuda.stream(stream):
        for _ in range(20):
            launch()
    torch.cuda.synchronize(dev)
    res = {k: {"rollout": [], "tiny": []} for k in makers}
    for _ in range(args.reps):   # alternate the methods
        for k, mk in makers.items():
            res[k]["rollout"].append(timed(launch, mk))
            res[k]["tiny"].append(timed(lambda: tiny.add_(1.0), mk))
    for k, r in res.items():
        med = statistics.median(r["rollout"])
        print(json.dumps({"method": k, "steps": args.steps, "envs": 65536, "rollout_ms_median": med,
                          "rollout_ms_min": min(r["rollout"]), "tiny_ms_median": statistics.median(r["tiny"]),
                          "env_steps_per_s": 65536 * args.steps / (med * 1e-3)}), flush=True)


if __name__ == "__main__":
    main()
