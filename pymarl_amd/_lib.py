"""ctypes binding of libmq_learner.so (the C ABI declared in include/mq_learner.h).

The product path has no fallback: if the library is missing, or the device is not a HIP GPU, the learner fails
loudly here. Build it with `python __graft_entry__.py build` (or `make -C pymarl_amd/csrc`).
"""
from __future__ import annotations

import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MQ_LEARNER_LIB", os.path.join(HERE, "lib", "libmq_learner.so"))

MIXER_NONE, MIXER_VDN, MIXER_QMIX = 0, 1, 2
NSUMS = 8
NSTATS = 8
PARAM_NAMES = [
    "fc1.weight", "fc1.bias", "rnn.weight_ih", "rnn.weight_hh", "rnn.bias_ih", "rnn.bias_hh", "fc2.weight",
    "fc2.bias", "hyper_w_1.weight", "hyper_w_1.bias", "hyper_w_final.weight", "hyper_w_final.bias",
    "hyper_b_1.weight", "hyper_b_1.bias", "V.0.weight", "V.0.bias", "V.2.weight", "V.2.bias",
]
P_COUNT = len(PARAM_NAMES)

# Every symbol include/mq_learner.h declares (checked by tests/test_boundary.py).
EXPORTS = [
    "mq_last_error", "mq_create", "mq_destroy", "mq_param_offsets", "mq_bind", "mq_forward_backward", "mq_apply",
    "mq_train_step", "mq_update_targets", "mq_copy_intermediate", "mq_mac_forward", "mq_agent_forward",
    "mq_greedy_actions", "mq_set_timing", "mq_phase_times", "mq_phase_names", "mq_set_data_parallel",
    "mq_last_plan", "mq_qmix_forward",
    # include/mc_coma.h
    "mc_create", "mc_destroy", "mc_param_offsets", "mc_bind", "mc_train_step", "mc_update_targets", "mc_policy",
    "mc_copy_intermediate", "mc_set_timing", "mc_phase_times", "mc_last_critic_path", "mq_comm_unique_id", "mq_comm_attach",
    "mq_comm_world", "mq_comm_detach", "mc_comm_attach", "mc_set_data_parallel", "mc_critic_forward",
    "mc_critic_forward_workspace", "mc_set_actor_shard", "mq_comm_use", "mq_comm_create", "mq_comm_free",
    "mc_comm_use", "mc_comm_detach",
]

# mc_allreduce_fn (include/mc_coma.h): int (*)(float* buf, int64_t count, void* stream, void* ctx)
MC_ALLREDUCE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p)

MC_P_COUNT = 6
MC_NTAIL = 8
MC_NSTATS = 16
COMA_STATS = ["critic_loss", "critic_grad_norm", "td_error_abs", "q_taken_mean", "target_mean", "advantage_mean",
              "coma_loss", "agent_grad_norm", "pi_max", "critic_steps", "mask_sum"]


class MQConfig(ctypes.Structure):
    _fields_ = [
        ("n_agents", ctypes.c_int32), ("n_actions", ctypes.c_int32), ("obs_dim", ctypes.c_int32),
        ("state_dim", ctypes.c_int32), ("rnn_hidden_dim", ctypes.c_int32), ("mixing_embed_dim", ctypes.c_int32),
        ("mixer", ctypes.c_int32), ("double_q", ctypes.c_int32), ("obs_last_action", ctypes.c_int32),
        ("obs_agent_id", ctypes.c_int32), ("gamma", ctypes.c_float), ("lr", ctypes.c_float),
        ("optim_alpha", ctypes.c_float), ("optim_eps", ctypes.c_float), ("grad_norm_clip", ctypes.c_float),
        ("max_batch", ctypes.c_int32), ("max_seq", ctypes.c_int32), ("huber_delta", ctypes.c_float),
    ]


class MQReplay(ctypes.Structure):
    _fields_ = [
        ("obs", ctypes.c_void_p), ("state", ctypes.c_void_p), ("actions", ctypes.c_void_p),
        ("avail_actions", ctypes.c_void_p), ("reward", ctypes.c_void_p), ("terminated", ctypes.c_void_p),
        ("filled", ctypes.c_void_p), ("ep_ids", ctypes.c_void_p), ("n_episodes", ctypes.c_int64),
        ("batch_size", ctypes.c_int32), ("t_len", ctypes.c_int32), ("t_stride", ctypes.c_int32),
        ("ep_ids_host", ctypes.c_void_p), ("avail_bits", ctypes.c_void_p),
    ]


class MCConfig(ctypes.Structure):
    _fields_ = [
        ("n_agents", ctypes.c_int32), ("n_actions", ctypes.c_int32), ("obs_dim", ctypes.c_int32),
        ("state_dim", ctypes.c_int32), ("rnn_hidden_dim", ctypes.c_int32), ("obs_last_action", ctypes.c_int32),
        ("obs_agent_id", ctypes.c_int32), ("mask_before_softmax", ctypes.c_int32), ("gamma", ctypes.c_float),
        ("td_lambda", ctypes.c_float), ("lr", ctypes.c_float), ("critic_lr", ctypes.c_float),
        ("optim_alpha", ctypes.c_float), ("optim_eps", ctypes.c_float), ("grad_norm_clip", ctypes.c_float),
        ("max_batch", ctypes.c_int32), ("max_seq", ctypes.c_int32),
    ]


class MQPlan(ctypes.Structure):
    _fields_ = [(k, ctypes.c_int32) for k in ("rows", "fused_fwd", "rw_fwd", "fused_bwd", "rw_bwd", "inline_ids",
                                               "hyper", "mix", "tiles", "dwh")]

    def as_dict(self):
        return {k: int(getattr(self, k)) for k, _ in self._fields_}


HYP_NAMES = {0: "none", 1: "ws", 2: "lds", 3: "gemm"}
MIX_NAMES = {0: "fast16", 1: "fast32", 2: "generic", 3: "stream"}

INLINE_IDS = 256   # MQ_INLINE_IDS: batches up to this size pass their episode ids in the kernel arguments
COMM_ID_BYTES = 128   # MQ_COMM_ID_BYTES (ncclUniqueId)


_LIB = None


class MQError(RuntimeError):
    pass


def load(required=True):
    """Load the shared library once; raise MQError (no fallback) if it cannot be loaded."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(LIB_PATH):
        if not required:
            return None
        raise MQError(f"libmq_learner.so not found at {LIB_PATH}; build it with `python __graft_entry__.py build`")
    import torch  # noqa: F401  (loads torch's HIP runtime first so the library binds to the same one)
    lib = ctypes.CDLL(LIB_PATH)
    vp, i32, i64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64
    sig = {
        "mq_last_error": ([], ctypes.c_char_p),
        "mq_phase_names": ([], ctypes.c_char_p),
        "mq_create": ([ctypes.POINTER(MQConfig), ctypes.POINTER(vp)], ctypes.c_int),
        "mq_destroy": ([vp], ctypes.c_int),
        "mq_param_offsets": ([vp, ctypes.POINTER(i64)], ctypes.c_int),
        "mq_bind": ([vp, vp, vp, vp, vp, vp, vp], ctypes.c_int),
        "mq_forward_backward": ([vp, ctypes.POINTER(MQReplay), vp], ctypes.c_int),
        "mq_apply": ([vp, vp], ctypes.c_int),
        "mq_train_step": ([vp, ctypes.POINTER(MQReplay), vp], ctypes.c_int),
        "mq_update_targets": ([vp, vp], ctypes.c_int),
        "mq_copy_intermediate": ([vp, ctypes.c_int, vp, ctypes.POINTER(i64), vp], ctypes.c_int),
        "mq_mac_forward": ([vp, ctypes.POINTER(MQReplay), i32, vp, vp, vp, i32, vp], ctypes.c_int),
        "mq_agent_forward": ([vp, vp, i32, vp, vp, vp, i32, vp], ctypes.c_int),
        "mq_greedy_actions": ([vp, vp, vp, i32, i32, vp], ctypes.c_int),
        "mq_set_timing": ([vp, i32, ctypes.c_uint32], ctypes.c_int),
        "mq_set_data_parallel": ([vp, i32], ctypes.c_int),
        "mq_last_plan": ([vp, ctypes.POINTER(MQPlan)], ctypes.c_int),
        "mq_qmix_forward": ([vp, i32, i32, i32, vp, vp, vp, i32, vp], ctypes.c_int),
        "mc_critic_forward_workspace": ([ctypes.POINTER(MCConfig), i32, i32], i64),
        "mc_critic_forward": ([vp, ctypes.POINTER(MCConfig), ctypes.POINTER(MQReplay), i32, vp, vp, vp], ctypes.c_int),
        "mq_phase_times": ([vp, ctypes.POINTER(ctypes.c_float), i32, ctypes.POINTER(i32)], ctypes.c_int),
        "mc_create": ([ctypes.POINTER(MCConfig), ctypes.POINTER(vp)], ctypes.c_int),
        "mc_destroy": ([vp], ctypes.c_int),
        "mc_param_offsets": ([vp, ctypes.POINTER(i64), ctypes.POINTER(i64)], ctypes.c_int),
        "mc_bind": ([vp, vp, vp, vp, vp, vp, vp, vp, vp], ctypes.c_int),
        "mc_train_step": ([vp, ctypes.POINTER(MQReplay), ctypes.c_float, vp], ctypes.c_int),
        "mc_update_targets": ([vp, vp], ctypes.c_int),
        "mc_policy": ([vp, vp, i32, i32, ctypes.c_float, i32, i32, vp], ctypes.c_int),
        "mc_copy_intermediate": ([vp, ctypes.c_int, vp, ctypes.POINTER(i64), vp], ctypes.c_int),
        "mc_set_timing": ([vp, i32], ctypes.c_int),
        "mc_phase_times": ([vp, ctypes.POINTER(ctypes.c_float)], ctypes.c_int),
        "mc_last_critic_path": ([vp], i32),
        "mq_comm_unique_id": ([vp], ctypes.c_int),
        "mq_comm_attach": ([vp, vp, i32, i32], ctypes.c_int),
        "mq_comm_world": ([vp], i32),
        "mq_comm_detach": ([vp], ctypes.c_int),
        "mc_comm_attach": ([vp, vp, i32, i32], ctypes.c_int),
        "mc_set_data_parallel": ([vp, MC_ALLREDUCE_FN, vp, i32, vp, i64], ctypes.c_int),
        "mc_set_actor_shard": ([vp, i32, i32], ctypes.c_int),
        "mq_comm_use": ([vp, vp], ctypes.c_int),
        "mq_comm_create": ([vp, i32, i32, ctypes.POINTER(vp)], ctypes.c_int),
        "mq_comm_free": ([vp], ctypes.c_int),
        "mc_comm_use": ([vp, vp], ctypes.c_int),
        "mc_comm_detach": ([vp], ctypes.c_int),
    }
    for name, (args, res) in sig.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = res
    _LIB = lib
    return lib


def check(rc):
    if rc != 0:
        msg = _LIB.mq_last_error().decode() if _LIB is not None else "library not loaded"
        if "not recognised" in msg:
            raise ValueError(msg)
        raise MQError(f"libmq_learner error {rc}: {msg}")


def ptr(t):
    """Device pointer of a torch tensor (None -> NULL)."""
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def stream_ptr(device=None):
    import torch
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def require_gpu(tensor_or_device):
    import torch
    dev = getattr(tensor_or_device, "device", tensor_or_device)
    dev = torch.device(dev)
    if dev.type != "cuda" or not torch.cuda.is_available():
        raise MQError(f"the MI355X learner path needs HIP device tensors (got device {dev}); there is no CPU "
                      "fallback — call .cuda() on the learner/MAC and keep the replay on the GPU")


class Handle:
    """RAII owner of an mq_handle."""

    def __init__(self, cfg: MQConfig):
        self.lib = load()
        h = ctypes.c_void_p()
        check(self.lib.mq_create(ctypes.byref(cfg), ctypes.byref(h)))
        self.h = h
        self.cfg = cfg
        offs = (ctypes.c_int64 * (P_COUNT + 1))()
        check(self.lib.mq_param_offsets(self.h, offs))
        self.offsets = list(offs)

    def __del__(self):
        try:
            if getattr(self, "h", None) and self.h.value:
                self.lib.mq_destroy(self.h)
                self.h = ctypes.c_void_p()
        except Exception:
            pass

    @property
    def n_params(self):
        return self.offsets[-1]


class ComaHandle:
    """RAII owner of an mc_handle (include/mc_coma.h)."""

    def __init__(self, cfg: MCConfig):
        self.lib = load()
        h = ctypes.c_void_p()
        check(self.lib.mc_create(ctypes.byref(cfg), ctypes.byref(h)))
        self.h = h
        self.cfg = cfg
        ao = (ctypes.c_int64 * (P_COUNT + 1))()
        co = (ctypes.c_int64 * (MC_P_COUNT + 1))()
        check(self.lib.mc_param_offsets(self.h, ao, co))
        self.agent_offsets = list(ao)
        self.critic_offsets = list(co)

    def __del__(self):
        try:
            if getattr(self, "h", None) and self.h.value:
                self.lib.mc_destroy(self.h)
                self.h = ctypes.c_void_p()
        except Exception:
            pass
