"""Device-resident A3C model + lockstep actor-learner workspace.

Replaces the reference's process-shared parameters (async.py:11-65:
RawArray-backed params and RMSProp `ms`, Hogwild writes) with ONE flat fp32
parameter buffer, one flat gradient buffer and one flat `ms` buffer in HBM,
laid out in Chainer namedparams order (a3c_ale.py:35,52) so checkpoints map
1:1 (HDF5 paths "0/0/W", ...).  PyTorch only allocates the memory; all
compute is in libasyncrl_hip.so.
"""
from __future__ import annotations

import ctypes
import weakref

import numpy as np
import torch

from ._lib import (ARCH_FF, ARCH_FF_NATURE, ARCH_LSTM, ARCH_RGB, ARCH_STACK, ARCH_STATES, ENV_GROUP_ALIGN, FWD_KEEP_STATE,
                   POOL_DONES, POOL_FRAMES, POOL_REWARDS, RESIZE_SCALAR, STAGE_HOST, STAGE_NAMES, check, lib, ptr,
                   stream_handle)


def param_shapes(arch: int, n_actions: int):
    """Chainer parameter shapes in link order (dqn_head.py:40-44,
    policy.py:49, v_function.py:25, Chainer L.LSTM upward/lateral; the
    Nature head dqn_head.py:16-20 with 512-wide policy / value heads; the
    RGB flag: NIPSDQNHead(n_input_channels=3), train_a3c_doom.py:28,46)."""
    c_in = 3 if arch & ARCH_RGB else 4
    arch &= ~(ARCH_RGB | ARCH_STACK | ARCH_STATES)
    if arch == ARCH_FF_NATURE:
        return [("0/0/W", (32, 4, 8, 8)), ("0/0/b", (32,)), ("0/1/W", (64, 32, 4, 4)), ("0/1/b", (64,)),
                ("0/2/W", (64, 64, 3, 3)), ("0/2/b", (64,)), ("0/3/W", (512, 3136)), ("0/3/b", (512,)),
                ("1/0/W", (n_actions, 512)), ("1/0/b", (n_actions,)), ("2/0/W", (1, 512)), ("2/0/b", (1,))]
    head = [("0/0/W", (16, c_in, 8, 8)), ("0/0/b", (16,)), ("0/1/W", (32, 16, 4, 4)), ("0/1/b", (32,)),
            ("0/2/W", (256, 2592)), ("0/2/b", (256,))]
    if arch == ARCH_FF:
        return head + [("1/0/W", (n_actions, 256)), ("1/0/b", (n_actions,)), ("2/0/W", (1, 256)),
                       ("2/0/b", (1,))]
    return head + [("1/upward/W", (1024, 256)), ("1/upward/b", (1024,)), ("1/lateral/W", (1024, 256)),
                   ("2/0/W", (n_actions, 256)), ("2/0/b", (n_actions,)), ("3/0/W", (1, 256)),
                   ("3/0/b", (1,))]


def init_like_torch(arch: int, n_actions: int, rng: np.random.Generator):
    """init_like_torch.py:5-22: U(+-1/sqrt(fan_in)) for every W and b
    (fan_in = in*kh*kw); host-side setup, not on the hot path."""
    shapes = dict(param_shapes(arch, n_actions))
    out = {}
    for name, shape in param_shapes(arch, n_actions):
        w = shapes[name.rsplit("/", 1)[0] + "/W"]
        stdv = 1.0 / np.sqrt(int(np.prod(w[1:])))
        out[name] = rng.uniform(-stdv, stdv, size=shape).astype(np.float32)
    return out



# every live DeviceNet, so a writer of a flat tensor can find the nets whose params it aliases
_NETS: "weakref.WeakSet[DeviceNet]" = weakref.WeakSet()


def nets_aliasing(t: torch.Tensor):
    """The live DeviceNets whose bound params overlap the memory of `t`."""
    if not isinstance(t, torch.Tensor) or t.device.type != "cuda":
        return []
    lo = t.data_ptr()
    hi = lo + t.numel() * t.element_size()
    out = []
    for n in list(_NETS):
        p = n._params
        b = p.data_ptr()
        if p.device == t.device and lo < b + p.numel() * p.element_size() and b < hi:
            out.append(n)
    return out


def check_pools(pool_len: int, *pools):
    """pool_len against each pool's leading dimension (the C ABI checks it
    again against the extents registered with arl_net_set_pool)."""
    if pool_len < 1:
        raise ValueError(f"pool_len must be >= 1, got {pool_len}")
    for p in pools:
        if p is not None and isinstance(p, torch.Tensor) and (p.dim() == 0 or p.shape[0] < pool_len):
            raise ValueError(f"pool_len {pool_len} exceeds a pool of shape {tuple(p.shape)}")

class DeviceNet:
    """One arl_net handle + the device memory it borrows."""

    def __init__(self, arch: int, n_actions: int, n_envs: int, t_max: int = 5, env_offset: int = 0,
                 seed: int = 0, device=None):
        self.device = torch.device(device if device is not None else "cuda")
        self.arch, self.n_actions, self.n_envs, self.t_max = arch, n_actions, n_envs, t_max
        self.rgb = bool(arch & ARCH_RGB)
        self.stack = bool(arch & ARCH_STACK)
        self.states = bool(arch & ARCH_STATES)
        self.base_arch = arch & ~(ARCH_RGB | ARCH_STACK | ARCH_STATES)
        self.env_offset, self.seed = env_offset, seed
        h = ctypes.c_void_p()
        check(lib.arl_net_create(ctypes.byref(h), arch, n_actions, n_envs, t_max, env_offset, seed),
              "arl_net_create")
        self._h = h
        P = lib.arl_net_param_floats(h)
        self.param_floats = P
        self._params = torch.zeros(P, dtype=torch.float32, device=self.device)
        self.grads = torch.zeros(P, dtype=torch.float32, device=self.device)
        self.ms = torch.zeros(P, dtype=torch.float32, device=self.device)
        self.workspace = torch.zeros(lib.arl_net_workspace_bytes(h), dtype=torch.uint8, device=self.device)
        check(lib.arl_net_bind(h, ptr(self._params), ptr(self.grads), ptr(self.ms), ptr(self.workspace)),
              "arl_net_bind")
        self._pver = self._params._version   # (binding bumped the net's parameter generation)
        _NETS.add(self)
        self.layout = {}
        shapes = dict(param_shapes(arch, n_actions))
        name = ctypes.create_string_buffer(64)
        for i in range(lib.arl_net_param_count(h)):
            off, num = ctypes.c_int64(), ctypes.c_int64()
            check(lib.arl_net_param_info(h, i, ctypes.byref(off), ctypes.byref(num), name, 64))
            key = name.value.decode()
            assert int(np.prod(shapes[key])) == num.value, key
            self.layout[key] = (off.value, shapes[key])
        self.n_params = sum(int(np.prod(s)) for _, s in self.layout.values())

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            lib.arl_net_destroy(h)
            self._h = None

    @property
    def handle(self):
        return self._h

    # ------------------------------------------------------------ params
    @property
    def params(self) -> torch.Tensor:
        """The bound flat f32 parameters (Chainer namedparams order).  In-place
        writes through this tensor or a view of it are seen (torch's version
        counter) and rebuild the FC weight planes before the next forward."""
        return self._params

    @params.setter
    def params(self, value) -> None:
        """net.params = x copies x into the bound memory (the C library keeps
        its pointer) and bumps the parameter generation."""
        self._params.copy_(torch.as_tensor(value, dtype=torch.float32, device=self.device).reshape(-1))
        self.params_changed()

    def _sync_params(self) -> None:
        """Bump the parameter generation if torch's version counter of the
        params moved since the last bump (an in-place write from Python)."""
        if self._params._version != self._pver:
            self.params_changed()

    def prepare(self, stream=None) -> None:
        """Make derived device state current on `stream` (arl_net_prepare):
        before env-range chains fork from it and before a graph replay."""
        self._sync_params()
        check(lib.arl_net_prepare(self._h, stream_handle(stream)), "arl_net_prepare")

    def param_generation(self):
        """(param_gen, planes_gen) of the C net: the planes are current iff equal."""
        a, b = ctypes.c_uint64(), ctypes.c_uint64()
        check(lib.arl_net_param_generation(self._h, ctypes.byref(a), ctypes.byref(b)), "arl_net_param_generation")
        return a.value, b.value

    def view(self, flat: torch.Tensor, name: str) -> torch.Tensor:
        off, shape = self.layout[name]
        return flat[off:off + int(np.prod(shape))].view(shape)

    def param(self, name: str) -> torch.Tensor:
        return self.view(self.params, name)

    def grad(self, name: str) -> torch.Tensor:
        return self.view(self.grads, name)

    def load_params(self, arrays: dict) -> None:
        for name, (off, shape) in self.layout.items():
            a = np.asarray(arrays[name], dtype=np.float32).reshape(shape)
            self.param(name).copy_(torch.from_numpy(a))
        self.params_changed()

    def params_changed(self) -> None:
        """Tell the net its params were written from outside (arl_net_params_changed):
        derived device state (the FC weight's split planes) is rebuilt before
        the next forward.  load_params / copy_params_from / the params setter /
        RMSpropAsync.update_arrays on these params call it; other in-place
        writes through the tensor are caught by its version counter."""
        check(lib.arl_net_params_changed(self._h), "arl_net_params_changed")
        self._pver = self._params._version

    def copy_params_from(self, other: "DeviceNet") -> None:
        """copy_param.copy_param (copy_param.py): this net's params <- other's."""
        self.params.copy_(other.params)
        self.params_changed()

    def state_dict(self, flat: torch.Tensor | None = None) -> dict:
        flat = self.params if flat is None else flat
        return {n: self.view(flat, n).detach().cpu().numpy().copy() for n in self.layout}

    # ------------------------------------------------------------ workspace
    def buffer(self, name: str, dtype=torch.uint8, shape=None) -> torch.Tensor:
        off, nb = ctypes.c_int64(), ctypes.c_int64()
        check(lib.arl_net_buffer(self._h, name.encode(), ctypes.byref(off), ctypes.byref(nb)), "arl_net_buffer")
        raw = self.workspace[off.value:off.value + nb.value]
        t = raw.view(dtype)
        return t.view(shape) if shape is not None else t

    # ------------------------------------------------------------ hot path
    def set_pools(self, frames=None, rewards=None, dones=None):
        """Register the input pools' extents with the net (arl_net_set_pool):
        the C ABI refuses an observation whose pools it does not know."""
        for kind, t in ((POOL_FRAMES, frames), (POOL_REWARDS, rewards), (POOL_DONES, dones)):
            if t is not None:
                check(lib.arl_net_set_pool(self._h, kind, ptr(t), t.numel() * t.element_size()), "arl_net_set_pool")

    def reset(self, stream=None):
        check(lib.arl_net_reset(self._h, stream_handle(stream)), "arl_net_reset")

    def observe(self, t: int, pair_pool: torch.Tensor, reward_pool=None, done_pool=None, pool_len: int = 1,
                force_reset: bool = False, resize_mode: int = RESIZE_SCALAR, stream=None, envs=None):
        """pair_pool: (pool_len, n, 2, 210, 160, 3) uint8 frame pairs; for an
        RGB net (arch | ARCH_RGB) the screens (pool_len, n, H, W, 3) instead.
        envs=(e0, ne): only envs [e0, e0 + ne) (arl_observe_envs)."""
        check_pools(pool_len, pair_pool, reward_pool, done_pool)
        self.set_pools(pair_pool, reward_pool, done_pool)
        if (self.stack or self.states) and envs is None:
            self.observe_stack(t, pair_pool, reward_pool, done_pool, pool_len, force_reset, stream)
            return
        if envs is not None:
            e0, ne = envs
            H, W = (pair_pool.shape[-3], pair_pool.shape[-2]) if self.rgb else (0, 0)
            check(lib.arl_observe_envs(self._h, t, e0, ne, ptr(pair_pool), H, W, ptr(reward_pool), ptr(done_pool),
                                       pool_len, int(force_reset), resize_mode, stream_handle(stream)),
                  "arl_observe_envs")
            return
        if self.rgb:
            H, W = pair_pool.shape[-3], pair_pool.shape[-2]
            check(lib.arl_observe_rgb(self._h, t, ptr(pair_pool), H, W, ptr(reward_pool), ptr(done_pool), pool_len,
                                      int(force_reset), resize_mode, stream_handle(stream)), "arl_observe_rgb")
            return
        check(lib.arl_observe(self._h, t, ptr(pair_pool), ptr(reward_pool), ptr(done_pool), pool_len,
                              int(force_reset), resize_mode, stream_handle(stream)), "arl_observe")

    def observe_stack(self, t: int, stack_pool=None, reward_pool=None, done_pool=None, pool_len: int = 1,
                      force_reset: bool = False, stream=None):
        """ARCH_STACK nets: stack_pool (pool_len, n, 4, 84, 84) uint8 whole
        frame stacks (arl_observe_stack); ARCH_STATES nets: (pool_len, n, 4,
        84, 84) f32 states, phi's output (arl_observe_states).  None ingests
        only the reward / done of step t (a terminal observation)."""
        check_pools(pool_len, stack_pool, reward_pool, done_pool)
        self.set_pools(stack_pool, reward_pool, done_pool)
        if self.states:
            if stack_pool is not None and stack_pool.dtype != torch.float32:
                raise ValueError("observe_stack: an ARCH_STATES net takes float32 states")
            check(lib.arl_observe_states(self._h, t, ptr(stack_pool), ptr(reward_pool), ptr(done_pool), pool_len,
                                         int(force_reset), stream_handle(stream)), "arl_observe_states")
            return
        check(lib.arl_observe_stack(self._h, t, ptr(stack_pool), ptr(reward_pool), ptr(done_pool), pool_len,
                                    int(force_reset), stream_handle(stream)), "arl_observe_stack")

    def truncate_window(self, t_len: int, stream=None):
        """Window steps [t_len, t_max) get no loss in the next learn (arl_truncate_window)."""
        check(lib.arl_truncate_window(self._h, t_len, stream_handle(stream)), "arl_truncate_window")

    def set_norm_fold(self, on: bool = True):
        """Fold the clip norm into learn()'s conv reduce (arl_net_set_norm_fold):
        only when the gradient is not all-reduced between learn and update."""
        check(lib.arl_net_set_norm_fold(self._h, int(on)), "arl_net_set_norm_fold")

    def set_returns_fusion(self, on: bool, gamma: float = 0.99, beta: float = 0.01, v_loss_coef: float = 0.5,
                           clip_reward: bool = True):
        """Run the learner's returns + heads backward inside the bootstrap
        step's policy launch (arl_net_set_returns_fusion; FF nets, one launch
        over all envs): the next act at t = t_max does them, and the window's
        LEARN_RETURNS part is skipped.  Bit-identical to the separate launch."""
        check(lib.arl_net_set_returns_fusion(self._h, int(on), gamma, beta, v_loss_coef, int(clip_reward)),
              "arl_net_set_returns_fusion")

    def set_loss(self, pi_loss_coef: float = 1.0, keep_loss_scale_same: bool = False):
        check(lib.arl_net_set_loss(self._h, pi_loss_coef, int(keep_loss_scale_same)), "arl_net_set_loss")

    def reset_state(self, e0: int = 0, n: int | None = None, stream=None):
        """LSTM: the pi_and_v recurrent state of rows [e0, e0 + n) -> None (arl_reset_state)."""
        n = self.n_envs - e0 if n is None else n
        check(lib.arl_reset_state(self._h, e0, n, stream_handle(stream)), "arl_reset_state")

    def act(self, t: int, mode: int = 1, stream=None, envs=None):
        """mode: 0 forward only, 1 sampled action, 2 greedy (first argmax);
        envs=(e0, ne): only envs [e0, e0 + ne) (arl_act_envs)."""
        self._sync_params()
        if envs is not None:
            check(lib.arl_act_envs(self._h, t, envs[0], envs[1], mode, stream_handle(stream)), "arl_act_envs")
            return
        check(lib.arl_act_mode(self._h, t, mode, stream_handle(stream)), "arl_act_mode")

    def observe_act(self, t: int, pair_pool: torch.Tensor, reward_pool=None, done_pool=None, pool_len: int = 1,
                    force_reset: bool = False, resize_mode: int = RESIZE_SCALAR, mode: int = 1, stream=None,
                    envs=None):
        """observe(t, ...) then act(t, mode) of envs (all if None).  (phi fused into the
        conv launch was built bit-identical and measured slower: DESIGN.md.)"""
        self.observe(t, pair_pool, reward_pool, done_pool, pool_len, force_reset, resize_mode, stream, envs)
        self.act(t, mode, stream, envs)

    def default_env_groups(self) -> int:
        """Forward chains per window that measured fastest on one MI355X:
        2 from 1,024 envs up, else 1.  Since the 512-env launches run two envs a
        conv workgroup and 64-row FC tiles, one chain of 512 envs beats two of
        256 (C4 0.497 vs 0.509-0.518 ms), while 1,024 LSTM envs still gain
        from two chains of 512 (profiles/r03/r3l)."""
        return 2 if self.n_envs >= 1024 else 1

    def env_groups(self, groups: int):
        """Split the envs into <= `groups` contiguous ranges (e0, ne) with e0 a
        multiple of ENV_GROUP_ALIGN; [(0, n_envs)] when they do not split."""
        if groups <= 1 or self.arch == ARCH_FF_NATURE or self.states:
            return [(0, self.n_envs)]
        per = -(-self.n_envs // groups)
        per = -(-per // ENV_GROUP_ALIGN) * ENV_GROUP_ALIGN
        out, e0 = [], 0
        while e0 < self.n_envs:
            ne = min(per, self.n_envs - e0)
            out.append((e0, ne))
            e0 += ne
        return out

    STAGES = {"conv_fwd": 1, "fc_fwd": 2, "policy": 3, "fc_bwd": 4, "conv_bwd": 5, "returns": 6, "conv_reduce": 7,
              "grad_sqnorm": 8, "lstm_gates": 9, "lstm_bptt": 10, "lstm_wgrad": 11, "rmsprop": 13}

    def run_stage(self, stage: str, t: int = 0, stream=None):
        """One window stage alone on the current workspace (timing / profiling)."""
        check(lib.arl_run_stage(self._h, self.STAGES[stage], t, stream_handle(stream)), "arl_run_stage")

    def learn(self, gamma=0.99, beta=1e-2, v_loss_coef=0.5, clip_reward=True, stream=None):
        """Gradient of the window (arl_learn)."""
        check(lib.arl_learn(self._h, gamma, beta, v_loss_coef, int(clip_reward), stream_handle(stream)), "arl_learn")

    def learn_parts(self, parts, gamma=0.99, beta=1e-2, v_loss_coef=0.5, clip_reward=True, stream=None):
        """arl_learn_part for each part in order on one stream (NIPS heads)."""
        h = stream_handle(stream)
        for p in parts:
            check(lib.arl_learn_part(self._h, p, gamma, beta, v_loss_coef, int(clip_reward), h), "arl_learn_part")

    def optimize(self, lr0=7e-4, total_steps=0, n_total=0, alpha=0.99, eps=0.1, clip=40.0, stream=None,
                 advance=False):
        """Clip + RMSProp; advance=True also ends the window (arl_optimize_advance)."""
        self._sync_params()
        if advance:
            check(lib.arl_optimize_advance(self._h, lr0, int(total_steps), int(n_total), alpha, eps, clip,
                                           stream_handle(stream)), "arl_optimize_advance")
        else:
            check(lib.arl_optimize(self._h, lr0, int(total_steps), int(n_total), alpha, eps, clip,
                                   stream_handle(stream)), "arl_optimize")

    def run_window(self, pair_pool, reward_pool, done_pool, pool_len: int, first: bool, resize_mode: int,
                   gamma: float, beta: float, v_loss_coef: float, clip_reward: bool, lr0: float, total_steps: int,
                   n_total: int, alpha: float, eps: float, clip: float, stream=None):
        """A whole lockstep window in one call (arl_run_window): T x (observe,
        act), the bootstrap, learn, clip + RMSProp and the advance -- the
        launches of observe / act / learn / optimize(advance=True) in order."""
        check_pools(pool_len, pair_pool, reward_pool, done_pool)
        self.set_pools(pair_pool, reward_pool, done_pool)
        self._sync_params()
        check(lib.arl_run_window(self._h, ptr(pair_pool), ptr(reward_pool), ptr(done_pool), pool_len, int(first),
                                 resize_mode, gamma, beta, v_loss_coef, int(clip_reward), lr0, int(total_steps),
                                 int(n_total), alpha, eps, clip, stream_handle(stream)), "arl_run_window")

    def advance(self, stream=None):
        check(lib.arl_advance(self._h, stream_handle(stream)), "arl_advance")

    def forward_states(self, states: torch.Tensor, mode: int = 0, stream=None, keep_same_state: bool = False):
        """pi_and_v on explicit f32 states into slot t_max (arl_forward_states);
        LSTM: advances the pi_and_v state unless keep_same_state."""
        n = states.shape[0]
        c = 3 if self.rgb else 4
        if states.dtype != torch.float32 or tuple(states.shape[1:]) != (c, 84, 84):
            raise ValueError(f"forward_states: need (n, {c}, 84, 84) float32 states")
        m = mode | (FWD_KEEP_STATE if keep_same_state else 0)
        self._sync_params()
        check(lib.arl_forward_states(self._h, ptr(states), n, m, stream_handle(stream)), "arl_forward_states")

    # ------------------------------------------------------------ window timeline (measurement)
    stamping = False

    def stamps_begin(self, cap: int):
        """From now on every stage launch records a timing event after its
        kernel(s) (arl_stamps_begin); read them with stamps_end()."""
        check(lib.arl_stamps_begin(self._h, int(cap)), "arl_stamps_begin")
        self.stamping = True

    def stamps_sparse(self, period: int):
        """Right after stamps_begin, for windows of `period` stamp calls: window w
        records only its calls t - 1 and t (t = w mod period; arl_stamps_sparse);
        stamps_end then gives ms = -1 for the intervals between unrelated calls."""
        check(lib.arl_stamps_sparse(self._h, int(period)), "arl_stamps_sparse")

    def stamp(self, stage: int = STAGE_HOST, stream=None):
        """A caller's stamp (e.g. after a collective); no-op unless stamping."""
        if self.stamping:
            check(lib.arl_stamp(self._h, int(stage), stream_handle(stream)), "arl_stamp")

    def stamps_end(self):
        """Stop the timeline; returns (ms, stages): ms[i] = time from stamp
        i - 1 to stamp i (ms[0] = 0), stages[i] = the stage name stamp i
        closes (arl_stamps_read; waits for the last stamp)."""
        self.stamping = False
        cnt = ctypes.c_int()
        check(lib.arl_stamps_end(self._h, ctypes.byref(cnt)), "arl_stamps_end")
        n = cnt.value
        ms = (ctypes.c_float * max(n, 1))()
        st = (ctypes.c_int * max(n, 1))()
        check(lib.arl_stamps_read(self._h, 0, n, ctypes.cast(ms, ctypes.c_void_p), ctypes.cast(st, ctypes.c_void_p)),
              "arl_stamps_read")
        return np.array(ms[:n], np.float64), [STAGE_NAMES.get(int(x), str(int(x))) for x in st[:n]]

    # ------------------------------------------------------------ outputs
    def step_outputs(self, t: int) -> dict:
        """Views of the policy / value outputs of window step t."""
        N, A, T1 = self.n_envs, self.n_actions, self.t_max + 1
        f32 = torch.float32
        return {
            "logits": self.buffer("logits", f32, (T1, N, A))[t],
            "probs": self.buffer("probs", f32, (T1, N, A))[t],
            "log_probs": self.buffer("logp", f32, (T1, N, A))[t],
            "v": self.buffer("v", f32, (T1, N))[t],
            "entropy": self.buffer("entropy", f32, (T1, N))[t],
            "actions": self.buffer("actions", torch.int32, (T1, N))[t],
            "action_log_probs": self.buffer("logp_a", f32, (T1, N))[t],
        }
