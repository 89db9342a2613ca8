"""ctypes binding of libasyncrl_hip.so (C ABI in include/asyncrl_hip.h).

torch is imported first on purpose: torch ships its own libamdhip64.so
(SONAME libamdhip64.so.7), so the extension resolves to the SAME HIP runtime
instance and torch's streams / device pointers are valid in our calls.

There is no fallback: if the shared object is missing the import fails loudly
(build it with `python -c "import __graft_entry__ as g; g.build()"` or
`make -C async-rl_amd/csrc`).
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (must precede the CDLL load, see module doc)

# ASYNCRL_HIP_LIB: alternative build of the same library (timing ablations only)
LIB_PATH = os.environ.get("ASYNCRL_HIP_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                                             "libasyncrl_hip.so")

if not os.path.exists(LIB_PATH):
    raise ImportError(
        f"asyncrl_amd: native extension not built ({LIB_PATH} missing); "
        "run `make -C async-rl_amd/csrc` or __graft_entry__.build()")

lib = ctypes.CDLL(LIB_PATH)

c_void_p = ctypes.c_void_p
c_int = ctypes.c_int
c_i64 = ctypes.c_int64
c_u64 = ctypes.c_uint64
c_double = ctypes.c_double

# name -> (restype, argtypes); every symbol declared in include/asyncrl_hip.h
SIGNATURES = {
    "arl_abi_version": (c_int, []),
    "arl_last_error": (ctypes.c_char_p, []),
    "arl_current_screen": (c_int, [c_void_p, c_void_p, c_void_p, c_i64, c_int, c_void_p]),
    "arl_max_luminance": (c_int, [c_void_p, c_void_p, c_void_p, c_i64, c_void_p]),
    "arl_phi_stack": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_i64, c_int, c_void_p]),
    "arl_dqn_phi": (c_int, [c_void_p, c_void_p, c_i64, c_void_p]),
    "arl_rgb_phi": (c_int, [c_void_p, c_i64, c_int, c_int, c_void_p, c_int, c_void_p]),
    "arl_net_create": (c_int, [ctypes.POINTER(c_void_p), c_int, c_int, c_int, c_int, c_int, c_u64]),
    "arl_net_destroy": (None, [c_void_p]),
    "arl_net_param_floats": (c_i64, [c_void_p]),
    "arl_net_param_count": (c_int, [c_void_p]),
    "arl_net_param_info": (c_int, [c_void_p, c_int, ctypes.POINTER(c_i64), ctypes.POINTER(c_i64),
                                   ctypes.c_char_p, c_int]),
    "arl_net_workspace_bytes": (c_i64, [c_void_p]),
    "arl_net_buffer": (c_int, [c_void_p, ctypes.c_char_p, ctypes.POINTER(c_i64), ctypes.POINTER(c_i64)]),
    "arl_net_bind": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "arl_net_reset": (c_int, [c_void_p, c_void_p]),
    "arl_net_params_changed": (c_int, [c_void_p]),
    "arl_net_prepare": (c_int, [c_void_p, c_void_p]),
    "arl_net_param_generation": (c_int, [c_void_p, ctypes.POINTER(c_u64), ctypes.POINTER(c_u64)]),
    "arl_net_set_pool": (c_int, [c_void_p, c_int, c_void_p, c_i64]),
    "arl_observe": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_i64, c_int, c_int, c_void_p]),
    "arl_observe_rgb": (c_int, [c_void_p, c_int, c_void_p, c_int, c_int, c_void_p, c_void_p, c_i64, c_int, c_int,
                                c_void_p]),
    "arl_observe_stack": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_i64, c_int, c_void_p]),
    "arl_observe_states": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_i64, c_int, c_void_p]),
    "arl_truncate_window": (c_int, [c_void_p, c_int, c_void_p]),
    "arl_net_set_loss": (c_int, [c_void_p, c_double, c_int]),
    "arl_net_set_norm_fold": (c_int, [c_void_p, c_int]),
    "arl_net_set_returns_fusion": (c_int, [c_void_p, c_int, c_double, c_double, c_double, c_int]),
    "arl_reset_state": (c_int, [c_void_p, c_i64, c_i64, c_void_p]),
    "arl_act": (c_int, [c_void_p, c_int, c_void_p]),
    "arl_act_mode": (c_int, [c_void_p, c_int, c_int, c_void_p]),
    "arl_observe_envs": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_int, c_int, c_void_p, c_void_p, c_i64,
                                 c_int, c_int, c_void_p]),
    "arl_act_envs": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p]),
    "arl_run_stage": (c_int, [c_void_p, c_int, c_int, c_void_p]),
    "arl_stamps_begin": (c_int, [c_void_p, c_int]),
    "arl_stamps_sparse": (c_int, [c_void_p, c_int]),
    "arl_stamp": (c_int, [c_void_p, c_int, c_void_p]),
    "arl_stamps_end": (c_int, [c_void_p, ctypes.POINTER(c_int)]),
    "arl_stamps_read": (c_int, [c_void_p, c_int, c_int, c_void_p, c_void_p]),
    "arl_learn": (c_int, [c_void_p, c_double, c_double, c_double, c_int, c_void_p]),
    "arl_run_window": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_i64, c_int, c_int, c_double, c_double,
                               c_double, c_int, c_double, c_i64, c_i64, c_double, c_double, c_double, c_void_p]),
    "arl_learn_part": (c_int, [c_void_p, c_int, c_double, c_double, c_double, c_int, c_void_p]),
    "arl_optimize": (c_int, [c_void_p, c_double, c_i64, c_i64, c_double, c_double, c_double, c_void_p]),
    "arl_advance": (c_int, [c_void_p, c_void_p]),
    "arl_optimize_advance": (c_int, [c_void_p, c_double, c_i64, c_i64, c_double, c_double, c_double, c_void_p]),
    "arl_forward_states": (c_int, [c_void_p, c_void_p, c_i64, c_int, c_void_p]),
    "arl_rmsprop": (c_int, [c_void_p, c_void_p, c_void_p, c_i64, c_double, c_double, c_double, c_double,
                            c_void_p, c_void_p]),
    "arl_policy": (c_int, [c_void_p, c_i64, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_u64, c_void_p,
                           c_i64, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                           c_void_p, c_void_p]),
    "arl_returns_lossgrad": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_i64,
                                     c_int, c_double, c_double, c_double, c_double, c_int, c_int, c_void_p,
                                     c_void_p, c_void_p, c_void_p]),
    "arl_stream_copy": (c_int, [c_void_p, c_void_p, c_i64, c_int, c_int, c_void_p]),
}

for _name, (_res, _args) in SIGNATURES.items():
    _fn = getattr(lib, _name)
    _fn.restype = _res
    _fn.argtypes = _args

if lib.arl_abi_version() != 4:
    raise ImportError(f"asyncrl_amd: {LIB_PATH} has ABI {lib.arl_abi_version()}, expected 4 (rebuild it)")

ARCH_FF = 0
ARCH_LSTM = 1
ARCH_FF_NATURE = 2   # A3CFF with NatureDQNHead (dqn_head.py:6-28)
ARCH_RGB = 16        # flag for FF / LSTM: the ViZDoom models (train_a3c_doom.py:25-63), RGB screens
ARCH_STACK = 32      # flag for FF / LSTM: observations are whole 4-screen stacks (ALE.state, ale.py:91-94)
ARCH_STATES = 64     # flag for FF / LSTM: observations are f32 (4, 84, 84) states, phi's output (a3c.py:34,73)
FWD_KEEP_STATE = 16  # arl_forward_states mode bit: LSTM keep_same_state (a3c_ale.py:57-60)
ABI_VERSION = 4
ACT_CONV_ONLY = 4      # arl_act_envs mode bits (env-group staggering)
ACT_AFTER_CONV = 8
ENV_GROUP_ALIGN = 32   # arl_observe_envs / arl_act_envs: e0 % ENV_GROUP_ALIGN == 0
LEARN_RETURNS, LEARN_TRUNK, LEARN_CONV = range(3)
POOL_FRAMES, POOL_REWARDS, POOL_DONES = range(3)   # arl_net_set_pool kinds
# window timeline stages (arl_stamps_*): arl_run_stage's 1..11, then the stamp-only ones
STAGE_NAMES = {1: "conv_fwd", 2: "fc_fwd", 3: "policy", 4: "fc_bwd", 5: "conv_bwd", 6: "returns", 7: "conv_reduce",
               8: "grad_sqnorm", 9: "lstm_gates", 10: "lstm_bptt", 11: "lstm_wgrad", 12: "phi", 13: "rmsprop",
               14: "lstm_cell", 15: "host", 16: "other"}
STAGE_HOST = 15
RESIZE_SCALAR = 0
RESIZE_SIMD = 1
RESIZE_CROP = 2      # flag, combine with SCALAR / SIMD: ale.py crop_or_scale='crop'


class ArlError(RuntimeError):
    pass


def check(rc: int, what: str = "") -> None:
    if rc != 0:
        msg = lib.arl_last_error().decode(errors="replace")
        raise ArlError(f"{what or 'asyncrl_hip'} failed (code {rc}): {msg}")


def ptr(t) -> int | None:
    """Device pointer of a torch tensor (None passes NULL)."""
    if t is None:
        return None
    if not t.is_cuda:
        raise ArlError("asyncrl_amd: tensors must live on the GPU (HIP device)")
    if not t.is_contiguous():
        raise ArlError("asyncrl_amd: tensors must be contiguous")
    return t.data_ptr()


def stream_handle(stream=None) -> int:
    s = stream if stream is not None else torch.cuda.current_stream()
    return s.cuda_stream
