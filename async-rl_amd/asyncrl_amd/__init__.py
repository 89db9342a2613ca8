"""asyncrl_amd -- MI355X-native batched A3C hot path (phi + forward + sample +
n-step update) behind the reference's A3C / dqn_phi / policy / RMSpropAsync
surfaces.  Compute lives in libasyncrl_hip.so (HIP, gfx950); see DESIGN.md."""
from ._lib import ARCH_FF, ARCH_FF_NATURE, ARCH_LSTM, ARCH_RGB, ARCH_STACK, ARCH_STATES, RESIZE_CROP, RESIZE_SCALAR, RESIZE_SIMD, ArlError, LIB_PATH  # noqa: F401
from .a3c import A3C, A3CFF, A3CFFNature, A3CLSTM, A3CModel, DoomA3CFF, DoomA3CLSTM  # noqa: F401
from .evaluation import eval_performance, run_episodes  # noqa: F401
from .dqn_phi import current_screen, dqn_phi, max_luminance, phi_stack, rgb_phi  # noqa: F401
from .net import DeviceNet, init_like_torch, param_shapes  # noqa: F401
from .policy_output import SoftmaxPolicyOutput, fc_softmax_policy_and_v  # noqa: F401
from .rmsprop_async import GradientClipping, RMSpropAsync  # noqa: F401
from . import serializers  # noqa: F401
from .hdf5 import read_hdf5, write_hdf5  # noqa: F401
