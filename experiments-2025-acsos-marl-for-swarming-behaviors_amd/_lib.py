"""ctypes binding of libswarm_hip.so (the C ABI declared in include/swarm_hip.h).

The shared library is built in-tree (``build.py``) and loaded after ``torch`` so
that it binds to the HIP runtime torch already loaded (same SONAME).  There is
no CPU fallback: if the library or a GPU is missing every call raises.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_float, c_int32, c_int64, c_uint32, c_uint64, c_void_p

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SWARM_LIB_PATH") or os.path.join(HERE, "libswarm_hip.so")

SWARM_GOTO, SWARM_OBSTACLE_AVOIDANCE, SWARM_FLOCKING = 0, 1, 2
GRAPH_COMPLETE, GRAPH_KNN, GRAPH_DENSE, GRAPH_RADIUS = 0, 1, 2, 3
CONV_GAT, CONV_GCN = 0, 1
F_SHARED_RESET, F_RANDOM_OA = 1, 2
N_PARAMS = 1673
NET_GCN, NET_GAT3 = 0, 1
GAT3_N_PARAMS = 409
GRAD_FLOATS = 1792        # SWARM_GRAD_FLOATS: gradient, loss sum, the clip norm's group partials
GRAD_SQ_BASE = 1680       # SWARM_GRAD_SQ_BASE
ADAM_F_NORM_PARTIALS = 1  # swarm_adam_cfg.flags
ERRORS = {-1: "SWARM_E_BADARG (invalid shape/config)",
          -2: "selected index k out of range (SWARM_E_KNN_K)",
          -3: "SWARM_E_NOGPU",
          -4: "SWARM_E_UNSUPPORTED (no fused-tick kernel for this configuration)"}
ABI_VERSION = 10


class SwarmConfig(ctypes.Structure):
    _fields_ = [("n_envs", c_int32), ("n_agents", c_int32), ("scenario", c_int32), ("graph", c_int32),
                ("knn_k", c_int32), ("conv", c_int32), ("env_offset", c_int32), ("flags", c_int32),
                ("seed", c_uint64), ("radius", c_float), ("net", c_int32)]


class SwarmReplay(ctypes.Structure):
    _fields_ = [("s", c_void_p), ("s_next", c_void_p), ("r", c_void_p), ("a", c_void_p),
                ("capacity", c_int32), ("pad", c_int32)]


class SwarmActOut(ctypes.Structure):
    _fields_ = [(n, c_void_p) for n in ("q", "actions", "reward", "obs", "avg_dist", "hits", "mult",
                                         "traj_pos", "traj_dist", "traj_hits")]


class SwarmAdamCfg(ctypes.Structure):
    _fields_ = [("lr", c_float), ("beta1", c_float), ("beta2", c_float), ("eps", c_float),
                ("max_norm", c_float), ("gamma", c_float), ("batch", c_int32),
                ("update_target_every", c_int32), ("world_size", c_int32), ("flags", c_int32),
                ("lr_d", ctypes.c_double), ("beta1_d", ctypes.c_double), ("beta2_d", ctypes.c_double)]


class SwarmLearner(ctypes.Structure):
    _fields_ = [(n, c_void_p) for n in ("w_cur", "w_nxt", "m_cur", "m_nxt", "v_cur", "v_nxt", "target", "grad")]


PEER_MAX = 8
PEER_HANDLE_BYTES = 64
PEER_SEQ_WORDS = 256


class SwarmPeer(ctypes.Structure):
    _fields_ = [("world_size", c_int32), ("rank", c_int32), ("recv", c_void_p * PEER_MAX), ("seq", c_void_p),
                ("err", c_void_p), ("timeout_us", c_uint32), ("pad", c_int32)]


# swarm_ctrl is 16 x 4-byte words on the device; field -> word index
CTRL_WORDS = 32
CTRL = dict(tick=0, write_slot=1, filled_slots=2, adam_step=3, eps=4, loss=5, grad_norm=6, trained=7, episode=8,
            adam_step_size=14, adam_inv_bc2=15, peer_hold=23, one_m_beta1=24, one_m_beta2=25)

_PROTOS = {
    "swarm_abi_version": (c_int32, []),
    "swarm_n_params": (c_int32, []),
    "swarm_build_info": (ctypes.c_char_p, []),
    "swarm_state_floats": (c_int64, [POINTER(SwarmConfig)]),
    "swarm_env_reset": (c_int32, [POINTER(SwarmConfig), c_void_p, c_uint32, c_void_p]),
    "swarm_env_sync_state": (c_int32, [POINTER(SwarmConfig), c_void_p, c_int32, c_void_p]),
    "swarm_env_step": (c_int32, [POINTER(SwarmConfig), c_void_p, c_void_p, POINTER(SwarmActOut), c_void_p]),
    "swarm_build_graph": (c_int32, [POINTER(SwarmConfig), c_void_p, c_void_p, c_void_p]),
    "swarm_edges_to_mult": (c_int32, [c_void_p, c_int64, c_int32, c_int32, c_void_p, c_void_p, c_void_p]),
    "swarm_q_forward": (c_int32, [POINTER(SwarmConfig), c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "swarm_act_step": (c_int32, [POINTER(SwarmConfig), c_void_p, c_void_p, POINTER(SwarmReplay), c_void_p,
                                 POINTER(SwarmActOut), c_void_p]),
    "swarm_train_act_step": (c_int32, [POINTER(SwarmConfig), POINTER(SwarmAdamCfg), POINTER(SwarmLearner), c_void_p,
                                       POINTER(SwarmReplay), c_void_p, POINTER(SwarmActOut), c_void_p, c_void_p]),
    "swarm_reduce_advance": (c_int32, [POINTER(SwarmConfig), POINTER(SwarmAdamCfg), c_void_p, POINTER(SwarmLearner),
                                       c_int32, c_void_p, c_void_p]),
    "swarm_sample_prepare": (c_int32, [POINTER(SwarmConfig), POINTER(SwarmAdamCfg), c_int32, c_void_p, c_void_p,
                                       c_void_p]),
    "swarm_adam_flush": (c_int32, [POINTER(SwarmConfig), POINTER(SwarmAdamCfg), POINTER(SwarmLearner), c_void_p,
                                   c_void_p]),
    "swarm_rollout": (c_int32, [POINTER(SwarmConfig), c_void_p, c_void_p, c_int32, c_uint32, c_float,
                                POINTER(SwarmActOut), c_void_p]),
    "swarm_td_workspace_floats": (c_int64, [POINTER(SwarmConfig), c_int32]),
    "swarm_td_grad": (c_int32, [POINTER(SwarmConfig), POINTER(SwarmAdamCfg), c_void_p, c_void_p,
                                POINTER(SwarmReplay), c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "swarm_grad_reduce": (c_int32, [POINTER(SwarmConfig), POINTER(SwarmAdamCfg), c_void_p, c_void_p, c_void_p]),
    "swarm_adam_step": (c_int32, [POINTER(SwarmConfig), POINTER(SwarmAdamCfg), c_void_p, c_void_p, c_void_p,
                                  c_void_p, c_void_p, c_int32, c_void_p, c_void_p]),
    "swarm_ctrl_init": (c_int32, [POINTER(SwarmAdamCfg), c_float, c_void_p, c_void_p]),
    "swarm_ctrl_advance": (c_int32, [POINTER(SwarmConfig), POINTER(SwarmReplay), c_void_p, c_void_p]),
    "swarm_host_topk_set": (c_int32, [POINTER(c_float), c_int32, c_int32, POINTER(ctypes.c_uint8)]),
    "swarm_train_tick_supported": (c_int32, [POINTER(SwarmConfig)]),
    "swarm_train_tick_workspace_bytes": (c_int64, [POINTER(SwarmConfig)]),
    "swarm_train_tick": (c_int32, [POINTER(SwarmConfig), POINTER(SwarmAdamCfg), POINTER(SwarmLearner), c_void_p,
                                   POINTER(SwarmReplay), c_void_p, POINTER(SwarmActOut), c_void_p, c_void_p,
                                   c_void_p, c_void_p]),
    "swarm_peer_buffer_bytes": (c_int64, []),
    "swarm_peer_alloc": (c_int32, [POINTER(c_void_p)]),
    "swarm_peer_free": (c_int32, [c_void_p]),
    "swarm_peer_ipc_handle": (c_int32, [c_void_p, c_void_p]),
    "swarm_peer_ipc_open": (c_int32, [c_void_p, POINTER(c_void_p)]),
    "swarm_peer_ipc_close": (c_int32, [c_void_p]),
    "swarm_reduce_advance_peer": (c_int32, [POINTER(SwarmConfig), POINTER(SwarmAdamCfg), c_void_p,
                                            POINTER(SwarmLearner), c_int32, c_void_p, POINTER(SwarmPeer), c_void_p]),
    "swarm_peer_allreduce": (c_int32, [POINTER(SwarmPeer), c_void_p, c_int32, c_void_p]),
    "swarm_host_sample_index": (c_uint32, [c_uint32, c_uint32, c_uint32, c_uint32, c_uint32]),
    "swarm_host_sample_position": (c_uint32, [c_uint32, c_uint32, c_uint32, c_uint32, c_uint32]),
}
EXPORTED = tuple(_PROTOS)

_lib = None


def load(require_gpu: bool = True):
    """Load the library (once).  Raises if it was not built or no GPU is visible."""
    global _lib
    if require_gpu and not torch.cuda.is_available():
        raise RuntimeError("libswarm_hip: no ROCm GPU visible (torch.cuda.is_available() is False); "
                           "this framework has no CPU fallback")
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"libswarm_hip.so not built at {LIB_PATH}; run __graft_entry__.build()")
        lib = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _PROTOS.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        if lib.swarm_abi_version() != ABI_VERSION:
            raise RuntimeError("libswarm_hip ABI mismatch")
        _lib = lib
    return _lib


def load_variant(path: str):
    """A second build of the library (e.g. build.HODROP_OUT, the hand-off overrun test
    library) with the same prototypes, loaded beside the main one; for tests."""
    if not os.path.exists(path):
        raise RuntimeError(f"{path} not built; run __graft_entry__.build()")
    lib = ctypes.CDLL(path)
    for name, (res, args) in _PROTOS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.swarm_abi_version() != ABI_VERSION:
        raise RuntimeError("libswarm_hip ABI mismatch")
    return lib


def check(rc: int, what: str):
    if rc != 0:
        msg = ERRORS.get(rc, f"hipError_t {rc}")
        raise RuntimeError(f"{what} failed: {msg}")


def ptr(t) -> int:
    return 0 if t is None else t.data_ptr()


def stream_ptr() -> int:
    return torch.cuda.current_stream().cuda_stream
