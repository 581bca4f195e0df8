"""ctypes binding of libpbn_env.so (include/pbn_env.h).

The HIP library is the only compute path: if it is missing or fails to load,
every entry point raises -- there is no CPU fallback.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from typing import Optional

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libpbn_env.so")
SRC_DIR = os.path.join(HERE, "csrc")
INCLUDE_DIR = os.path.join(HERE, "..", "include")

MODE_AUTORESET = 1
MODE_RANDOM_ACTIONS = 2
FLAG_TERMINATED = 1
FLAG_TRUNCATED = 2
FLAG_IN_ATTRACTOR = 4
FLAG_PERTURBED = 8
FLAG_RESET = 16
FLAG_UNSETTLED = 32

EXPORTS = ["pbn_net_create", "pbn_net_destroy", "pbn_net_words", "pbn_reset", "pbn_step", "pbn_step_dev", "pbn_step_dev_store",
           "pbn_rollout", "pbn_rollout_ex", "pbn_state_histogram", "pbn_obs_unpack", "pbn_bilinear_targets", "pbn_q_to_flipmask",
           "pbn_q_to_flipmask_dev",
           "pbn_heads_to_flipmask", "pbn_qnet_heads", "pbn_qnet_flipmask", "pbn_qnet_heads_from_state",
           "pbn_qnet_flipmask_from_state", "pbn_replay_store", "pbn_replay_advance", "pbn_replay_batch", "pbn_bdq_td_loss", "pbn_bdq_layout", "pbn_bdq_learn_workspace",
           "pbn_bdq_pack", "pbn_bdq_image_floats", "pbn_bdq_learn", "pbn_copy_async", "pbn_rollout_copy", "pbn_host_buffer", "pbn_host_buffer_free", "pbn_stream_sync",
           "pbn_last_error", "pbn_abi_version"]
SOURCES = ["pbn_env.hip", "pbn_settle.hip", "pbn_agent.hip", "pbn_qnet.hip", "pbn_learn.hip"]

_lib: Optional[ctypes.CDLL] = None


class PbnError(RuntimeError):
    pass


class RingStore(ctypes.Structure):
    """pbn_ring_store (include/pbn_env.h, ABI 11): the replay ring pbn_step_dev_store writes the
    step's transitions into (pbn_replay_store's layout)."""
    _fields_ = [("capacity", ctypes.c_int64), ("d_pos", ctypes.c_void_p), ("d_state", ctypes.c_void_p),
                ("d_next_state", ctypes.c_void_p), ("d_target", ctypes.c_void_p), ("d_action", ctypes.c_void_p),
                ("d_reward", ctypes.c_void_p), ("d_done", ctypes.c_void_p), ("d_actions_in", ctypes.c_void_p),
                ("n_branches", ctypes.c_int32), ("done_mask", ctypes.c_uint32), ("d_done_out", ctypes.c_void_p)]


class FrameAdvance(ctypes.Structure):
    """pbn_frame_advance (include/pbn_env.h, ABI 9): the counters a captured learning frame's fused
    update advances in its last launch, and the next frame's replay rows it draws."""
    _fields_ = [("n_store", ctypes.c_int64), ("capacity", ctypes.c_int64), ("d_pos", ctypes.c_void_p),
                ("d_size", ctypes.c_void_p), ("d_step", ctypes.c_void_p), ("d_eps64", ctypes.c_void_p),
                ("d_eps32", ctypes.c_void_p), ("eps_final", ctypes.c_double), ("eps_step", ctypes.c_double),
                ("n_idx", ctypes.c_int64), ("seed", ctypes.c_uint64), ("d_counter", ctypes.c_void_p),
                ("d_idx", ctypes.c_void_p)]


def build(verbose: bool = False, out: str = LIB_PATH, defines=()) -> str:
    """Compile csrc/*.hip for gfx950 into pbn_rl_amd/libpbn_env.so (in-tree): one object per
    source, compiled in parallel, then one link.  ``defines`` builds a diagnostic variant (e.g.
    PBN_STAMPS) into another path."""
    import tempfile
    flags = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-Wno-unused-result",
             *[f"-D{d}" for d in defines]]
    with tempfile.TemporaryDirectory(prefix="pbn_build_") as tmp:
        objs, procs = [], []
        for f in SOURCES:
            obj = os.path.join(tmp, f.replace(".hip", ".o"))
            cmd = ["hipcc", *flags, "-c", "-o", obj, os.path.join(SRC_DIR, f)]
            if verbose:
                print(" ".join(cmd))
            procs.append((subprocess.Popen(cmd), cmd))
            objs.append(obj)
        rcs = [(p.wait(), cmd) for p, cmd in procs]   # all of them, before the directory goes
        for rc, cmd in rcs:
            if rc != 0:
                raise subprocess.CalledProcessError(rc, cmd)
        cmd = ["hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o", out + ".tmp", *objs]
        if verbose:
            print(" ".join(cmd))
        subprocess.run(cmd, check=True)
    os.replace(out + ".tmp", out)
    return out


def load() -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    path = os.environ.get("PBN_LIB", LIB_PATH)  # diagnostic builds only
    if not os.path.exists(path):
        raise PbnError(f"{path} not built: run `python -c 'import __graft_entry__ as g; g.build()'`")
    L = ctypes.CDLL(path)
    vp, u64, i64, u32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int64, ctypes.c_uint32
    L.pbn_net_create.argtypes = [vp, ctypes.POINTER(vp)]
    L.pbn_net_create.restype = ctypes.c_int
    L.pbn_net_destroy.argtypes = [vp]
    L.pbn_net_destroy.restype = ctypes.c_int
    L.pbn_net_words.argtypes = [vp]
    L.pbn_net_words.restype = ctypes.c_int
    L.pbn_reset.argtypes = [vp, u64, u64, u64, i64, vp, vp, vp, vp]
    L.pbn_reset.restype = ctypes.c_int
    L.pbn_step.argtypes = [vp, u64, u64, u64, i64, u32, vp, vp, vp, vp, vp, vp, vp, vp, vp]
    L.pbn_step.restype = ctypes.c_int
    L.pbn_step_dev.argtypes = [vp, u64, vp, u64, i64, u32, vp, vp, vp, vp, vp, vp, vp, vp, vp]
    L.pbn_step_dev.restype = ctypes.c_int
    if hasattr(L, "pbn_step_dev_store"):   # (ABI 11)
        L.pbn_step_dev_store.argtypes = [vp, u64, vp, u64, i64, u32, vp, vp, vp, vp, vp, vp, vp, vp, vp]
        L.pbn_step_dev_store.restype = ctypes.c_int
    L.pbn_rollout.argtypes = [vp, u64, u64, u64, i64, ctypes.c_int32, u32, vp, vp, vp, vp, vp, vp, vp, vp, vp]
    L.pbn_rollout.restype = ctypes.c_int
    L.pbn_rollout_ex.argtypes = [vp, u64, u64, u64, i64, ctypes.c_int32, u32, vp, vp, vp, vp, vp, vp, vp, vp, vp,
                                 vp]
    L.pbn_rollout_ex.restype = ctypes.c_int
    L.pbn_state_histogram.argtypes = [vp, i64, i64, i64, ctypes.c_int32, vp, vp]
    L.pbn_state_histogram.restype = ctypes.c_int
    L.pbn_obs_unpack.argtypes = [vp, i64, vp, vp, vp, vp]
    L.pbn_obs_unpack.restype = ctypes.c_int
    L.pbn_bilinear_targets.argtypes = [vp, i64, vp, vp, vp, vp, ctypes.c_int32, ctypes.c_int32, ctypes.c_float,
                                       vp, vp]
    L.pbn_bilinear_targets.restype = ctypes.c_int
    L.pbn_q_to_flipmask.argtypes = [vp, u64, u64, u64, i64, ctypes.c_int32, ctypes.c_int32, vp, ctypes.c_float,
                                    vp, vp, vp]
    L.pbn_q_to_flipmask.restype = ctypes.c_int
    L.pbn_q_to_flipmask_dev.argtypes = [vp, u64, vp, u64, i64, ctypes.c_int32, ctypes.c_int32, vp, ctypes.c_float,
                                        vp, vp, vp, vp]
    L.pbn_q_to_flipmask_dev.restype = ctypes.c_int
    L.pbn_heads_to_flipmask.argtypes = [vp, u64, u64, vp, u64, i64, ctypes.c_int32, ctypes.c_int32, vp, ctypes.c_float,
                                        vp, vp, vp, vp]
    L.pbn_heads_to_flipmask.restype = ctypes.c_int
    L.pbn_qnet_heads.argtypes = [vp, i64] + [vp] * 11 + [ctypes.c_int32, ctypes.c_int32, ctypes.c_float, vp, vp]
    L.pbn_qnet_heads.restype = ctypes.c_int
    L.pbn_qnet_flipmask.argtypes = ([vp, u64, u64, vp, u64, i64] + [vp] * 11 +
                                    [ctypes.c_int32, ctypes.c_int32, ctypes.c_float, ctypes.c_float, vp, vp, vp, vp])
    L.pbn_qnet_flipmask.restype = ctypes.c_int
    L.pbn_qnet_heads_from_state.argtypes = [vp, i64] + [vp] * 14 + [ctypes.c_int32, ctypes.c_int32, ctypes.c_float,
                                                                     vp, vp]
    L.pbn_qnet_heads_from_state.restype = ctypes.c_int
    L.pbn_qnet_flipmask_from_state.argtypes = ([vp, u64, u64, vp, u64, i64] + [vp] * 14 +
                                               [ctypes.c_int32, ctypes.c_int32, ctypes.c_float, ctypes.c_float,
                                                vp, vp, vp, vp])
    L.pbn_qnet_flipmask_from_state.restype = ctypes.c_int
    L.pbn_last_error.argtypes = []
    L.pbn_last_error.restype = ctypes.c_char_p
    L.pbn_replay_store.argtypes = ([i64, vp, i64, ctypes.c_int32, ctypes.c_int32] + [vp] * 6 + [u32, vp] + [vp] * 6 +
                                   [vp] * 4 + [vp])
    L.pbn_replay_store.restype = ctypes.c_int
    L.pbn_replay_batch.argtypes = [vp, i64, vp, i64, vp, vp, vp, vp, ctypes.c_int32, vp, vp, vp, vp, vp, vp, vp]
    L.pbn_replay_batch.restype = ctypes.c_int
    L.pbn_bdq_td_loss.argtypes = [vp, vp, vp, vp, vp, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_float,
                                  vp, vp, vp, vp]
    L.pbn_bdq_td_loss.restype = ctypes.c_int
    i32, f32 = ctypes.c_int32, ctypes.c_float
    if hasattr(L, "pbn_bdq_learn"):   # (diagnostic builds of older revisions predate the fused update)
        L.pbn_replay_advance.argtypes = [i64, i64, vp, vp, vp, vp, vp, ctypes.c_double, ctypes.c_double, i64, u64,
                                         vp, vp, vp]
        L.pbn_replay_advance.restype = ctypes.c_int
        L.pbn_bdq_layout.argtypes = [i32, i32, vp]
        L.pbn_bdq_layout.restype = ctypes.c_int
        L.pbn_bdq_learn_workspace.argtypes = [i32, i32, i64, vp]
        L.pbn_bdq_learn_workspace.restype = ctypes.c_int
        L.pbn_bdq_pack.argtypes = [vp, i32, vp, vp, vp]
        L.pbn_bdq_pack.restype = ctypes.c_int
        if hasattr(L, "pbn_bdq_image_floats"):   # (ABI 10)
            L.pbn_bdq_image_floats.argtypes = [vp, i32, vp]
            L.pbn_bdq_image_floats.restype = ctypes.c_int
        L.pbn_bdq_learn.argtypes = ([vp, i64, vp, i64, vp, vp, vp, vp, i32, vp, vp] + [vp] * 7 + [f32] * 7 +
                                    [vp, i64, vp, vp, vp, vp])
        L.pbn_bdq_learn.restype = ctypes.c_int
    L.pbn_copy_async.argtypes = [vp, vp, i64, vp]
    L.pbn_copy_async.restype = ctypes.c_int
    L.pbn_rollout_copy.argtypes = [vp, u64, u64, u64, i64, ctypes.c_int32, u32, vp, vp, vp, vp, vp, vp, vp, vp, vp,
                                   vp, vp, i64, vp]
    L.pbn_rollout_copy.restype = ctypes.c_int
    if hasattr(L, "pbn_host_buffer"):   # (ABI 9)
        L.pbn_host_buffer.argtypes = [i64, ctypes.POINTER(vp), ctypes.POINTER(vp)]
        L.pbn_host_buffer.restype = ctypes.c_int
        L.pbn_host_buffer_free.argtypes = [vp]
        L.pbn_host_buffer_free.restype = ctypes.c_int
        L.pbn_stream_sync.argtypes = [vp]
        L.pbn_stream_sync.restype = ctypes.c_int
    L.pbn_abi_version.argtypes = []
    L.pbn_abi_version.restype = ctypes.c_int
    _lib = L
    return L


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = load().pbn_last_error().decode(errors="replace")
        raise PbnError(f"{what} failed ({rc}): {msg}")


class NetHandle:
    """Owns one pbn_net (device tables) on the current device."""

    def __init__(self, spec):
        L = load()
        self.spec = spec
        h = ctypes.c_void_p()
        check(L.pbn_net_create(ctypes.addressof(spec.desc), ctypes.byref(h)), "pbn_net_create")
        self.handle = h
        self.words = L.pbn_net_words(h)

    def close(self) -> None:
        if getattr(self, "handle", None) is not None and self.handle.value:
            load().pbn_net_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
