"""A3C agent and models on the MI355X hot path (drop-in for a3c.py / a3c_ale.py).

Reference surfaces kept: `A3CModel` (a3c.py:15-24: pi_and_v, reset_state,
unchain_backward), `A3CFF` / `A3CLSTM` (a3c_ale.py:28-70), `A3C` (a3c.py:27-185:
__init__ arguments, act(state, reward, is_state_terminal), sync_parameters,
load_model / save_model).

Two ways in, one set of kernels:

* `A3C.act(state, reward, is_state_terminal) -> int | None` on a one-env model
  (the default for n_envs = 1) is the reference's contract call for call
  (a3c.py:67-167).  The model sees phi(state) (a3c.py:73; phi is the identity
  by default, a3c.py:34): with phi = asyncrl_amd.dqn_phi, `state` is ALE.state
  (4 uint8 84x84 screens, ale.py:91-94), kept as uint8 and scaled by the conv
  kernels (bit-exact dqn_phi); with any other phi (or none) the float32
  (4, 84, 84) value phi returns is the conv input (an ARCH_STATES ring).  The
  window restarts at every update (t_start = t, a3c.py:152); a terminal call
  runs the R = 0 update over the steps since the last one, resets the
  recurrent state and returns None (a3c.py:77-83,165-167); a full window
  bootstraps with v(s) at pre-update parameters and acts on s with the
  post-update ones (a3c.py:85,156); pi_loss_coef, v_loss_coef and
  keep_loss_scale_same scale the losses as at a3c.py:110-121.  The frames
  live in an ARCH_STACK (uint8) or ARCH_STATES (f32) ring, one whole stack
  per slot; the update is the same device learner as the batched path,
  restricted to the window's steps (arl_truncate_window).

* `A3C.act_batch(pairs, reward, is_state_terminal)` / `run_window(...)` on an
  n-env model: the envs step in lockstep, phi runs on the GPU
  from raw frame pairs, and every t_max steps one update is made from the SUM
  of all envs' window-segment gradients at fixed parameters (a terminal
  inside a window closes that env's segment with R = 0, exactly like
  a3c.py:82-83), all-reduced over ranks with RCCL when torch.distributed is
  initialised, then clipped and applied by RMSpropAsync.  Hogwild races are
  gone; replicas stay bitwise identical.  batch_loss="mean" divides the
  summed loss by the envs of all ranks (effective step size).
  Batched convention: a terminal env's observation is already the first
  frame of its next episode (auto-reset).
"""
from __future__ import annotations

import os

import numpy as np
import torch

from ._lib import (ACT_AFTER_CONV, ACT_CONV_ONLY, ARCH_FF, ARCH_FF_NATURE, ARCH_LSTM, ARCH_RGB, ARCH_STACK,
                   ARCH_STATES, LEARN_CONV, RESIZE_SCALAR)
from .dqn_phi import dqn_phi as _device_dqn_phi
from .distributed import allreduce_grads, dist_initialized, world_info
from .net import DeviceNet, init_like_torch
from . import serializers
from .policy_output import SoftmaxPolicyOutput

# > 1 rank: split the gradient all-reduce around the conv backward (ARL_OVERLAP_ALLREDUCE=0: one call,
# the A arm of the 2-rank rehearsal)
OVERLAP_ALLREDUCE = os.environ.get("ARL_OVERLAP_ALLREDUCE", "1") != "0"
# a single-chain window without collectives as one C call (arl_run_window: the same launches without a
# host round trip per step); ARL_WINDOW_C=0 issues them step by step from Python (the A arm)
WINDOW_C = os.environ.get("ARL_WINDOW_C", "1") != "0"
# the step-by-step FF window runs the learner's returns inside the bootstrap policy launch, as the C
# window does; ARL_FUSE_RETURNS=0 keeps the separate returns launch (the bitwise arm of
# test_conv_fwd_two_envs_identical)
FUSE_RETURNS = os.environ.get("ARL_FUSE_RETURNS", "1") != "0"

def _is_dqn_phi(phi) -> bool:
    """phi IS dqn_phi (dqn_phi.py:4-17): this package's function object, or the
    reference module's own (module dqn_phi, qualified name dqn_phi).  Its
    output is the uint8 screens / 255, which the conv kernels apply
    bit-exactly, so the ring keeps the uint8 screens.  Matched by identity
    only: a wrapper, partial or look-alike of the same name may change the
    output, so it takes the general path (phi's f32 output on an
    ARCH_STATES ring), which is always exact."""
    if phi is _device_dqn_phi:
        return True
    return (callable(phi) and getattr(phi, "__module__", None) == "dqn_phi"
            and getattr(phi, "__qualname__", None) == "dqn_phi" and not hasattr(phi, "__wrapped__"))


def _to_device_f32(state, device) -> torch.Tensor:
    t = state if torch.is_tensor(state) else torch.from_numpy(np.ascontiguousarray(np.asarray(state, np.float32)))
    t = t.to(device=device, dtype=torch.float32)
    if t.dim() == 3:
        t = t.unsqueeze(0)
    return t.contiguous()


class A3CModel:
    """a3c.py:15-24.

    frames: "stacks" -- observations are whole ALE.state stacks (the A3C.act
    drop-in with phi = dqn_phi; default for n_envs = 1), "states" -- float32
    (4, 84, 84) states, whatever A3C's phi plugin returns (A3C switches a
    one-env model to it for any phi but asyncrl_amd.dqn_phi), or "pairs" --
    raw (frame 4, frame 3) pairs whose phi runs on the GPU (the batched hot
    path; default for n_envs > 1).  RGB (Doom) and Nature models take their
    own inputs."""

    arch = ARCH_FF

    def __init__(self, n_actions: int, n_envs: int = 1, t_max: int = 5, seed: int = 0, env_offset: int = 0,
                 init_seed: int | None = 0, device=None, frames: str | None = None):
        self.n_actions = n_actions
        arch = self.arch
        stackable = arch in (ARCH_FF, ARCH_LSTM)
        if frames is None:
            frames = "stacks" if (n_envs == 1 and stackable) else "pairs"
        if frames not in ("stacks", "states", "pairs"):
            raise ValueError("frames must be 'stacks', 'states' or 'pairs'")
        if frames != "pairs" and not stackable:
            raise ValueError(f"frames={frames!r} applies to the NIPS-head FF / LSTM models")
        arch |= {"stacks": ARCH_STACK, "states": ARCH_STATES, "pairs": 0}[frames]
        self.frames = frames
        self.net = DeviceNet(arch, n_actions, n_envs, t_max, env_offset=env_offset, seed=seed, device=device)
        if init_seed is not None:
            self.net.load_params(init_like_torch(self.arch, n_actions, np.random.default_rng(init_seed)))

    def set_frames(self, frames: str):
        """Rebuild the device net for another observation layout ("stacks"
        / "states"), keeping the parameters and the RMSProp statistics.  Only
        before an agent binds the model: an A3C holds the net it was built
        with, so a later switch would leave it stepping parameters the
        optimizer no longer updates."""
        if frames == self.frames:
            return
        if frames not in ("stacks", "states") or self.frames not in ("stacks", "states"):
            raise ValueError("set_frames switches between 'stacks' and 'states' only")
        if getattr(self, "_bound", False):
            raise ValueError(f"set_frames({frames!r}): an A3C agent already runs this model with frames="
                             f"{self.frames!r}; pick the layout (the phi plugin) before the first agent binds it, "
                             "or give the second agent its own model")
        old = self.net
        arch = self.arch | (ARCH_STACK if frames == "stacks" else ARCH_STATES)
        net = DeviceNet(arch, self.n_actions, old.n_envs, old.t_max, env_offset=old.env_offset, seed=old.seed,
                        device=old.device)
        net.copy_params_from(old)
        net.ms.copy_(old.ms)
        self.net, self.frames = net, frames

    def pi_and_v(self, state, keep_same_state: bool = False, deterministic: bool = False):
        """a3c_ale.py:38-40 / 55-63: state (n, C, 84, 84) float32 (dqn_phi
        output; a device tensor, or host data that is uploaded), n <=
        n_envs.  The policy output is computed eagerly: action_indices holds
        a Philox draw (a fresh one per call), or, with deterministic=True,
        most_probable_actions holds the first argmax (the two eval modes of
        a3c_ale.py:73-89).  LSTM models carry their pi_and_v recurrent state
        across calls (reset_state() clears it; keep_same_state=True leaves it
        as it was, a3c_ale.py:57-60).  The returned tensors are copies."""
        x = _to_device_f32(state, self.net.device)
        mode = 2 if deterministic else 1
        self.net.forward_states(x, mode=mode, keep_same_state=keep_same_state)
        n = x.shape[0]
        o = {k: v[:n].clone() for k, v in self.net.step_outputs(self.net.t_max).items()}
        return SoftmaxPolicyOutput(o, greedy=deterministic), o["v"]

    def reset_state(self):
        """a3c_ale.py:65-66: the pi_and_v recurrent state -> None (LSTM; a
        no-op for FF).  The lockstep window's state is reset by terminals."""
        self.net.reset_state()

    def unchain_backward(self):
        """a3c_ale.py:68-70: nothing to cut -- the device learner's BPTT is
        truncated at every window edge by construction."""

    def namedparams(self):
        return self.net.state_dict()


class A3CFF(A3CModel):
    """a3c_ale.py:28-40: NIPSDQNHead -> FCSoftmaxPolicy + FCVFunction."""
    arch = ARCH_FF


class A3CFFNature(A3CModel):
    """A3CFF (a3c_ale.py:28-40) with dqn_head.NatureDQNHead (dqn_head.py:6-28:
    conv 4->32 k8 s4, 32->64 k4 s2, 64->64 k3 s1, Linear 3136->512) and
    FCSoftmaxPolicy(512, A) / FCVFunction(512).  Parameters keep the Chainer
    link paths: 0/0..0/3 (head), 1/0 (policy), 2/0 (value)."""
    arch = ARCH_FF_NATURE


class A3CLSTM(A3CModel):
    """a3c_ale.py:43-70: NIPSDQNHead -> L.LSTM(256, 256) -> policy + value."""
    arch = ARCH_LSTM


class DoomA3CFF(A3CModel):
    """train_a3c_doom.py:25-38 A3CFF: NIPSDQNHead(n_input_channels=3) on the
    RGB screen (phi = train_a3c_doom.py:21-23, no frame stack) ->
    FCSoftmaxPolicy + FCVFunction.  pi_and_v takes rgb_phi output
    (n, 3, 84, 84); A3C.act_batch takes the raw (n, H, W, 3) screens."""
    arch = ARCH_FF | ARCH_RGB


class DoomA3CLSTM(A3CModel):
    """train_a3c_doom.py:41-63 A3CLSTM: the RGB NIPS head -> L.LSTM(256, 256)
    -> policy + value."""
    arch = ARCH_LSTM | ARCH_RGB


class A3C:
    """a3c.py:27-185.  On a one-env model `act` is the reference's call (one
    env-step, int | None); on an n-env model one `act_batch` call is one
    env-step of all envs and every t_max calls also performs the update."""

    def __init__(self, model: A3CModel, optimizer, t_max: int, gamma: float, beta: float = 1e-2,
                 process_idx: int = 0, clip_reward: bool = True, phi=None, pi_loss_coef: float = 1.0,
                 v_loss_coef: float = 0.5, keep_loss_scale_same: bool = False, resize_mode: int = RESIZE_SCALAR,
                 process_group=None, batch_loss: str = "sum", collectives: bool | None = None):
        """collectives: all-reduce the window gradient over the process group
        (default: when torch.distributed is initialised with > 1 rank; True
        also on a one-rank group, which runs the RCCL calls of the N > 1 path
        on one GPU).  A one-env drop-in model (the reference-contract `act`)
        updates at its own episode's terminals, so its ranks would enter the
        collectives at different times: it refuses collectives, and with
        collectives=False every rank is an independent learner."""
        if model.net.t_max != t_max:
            raise ValueError("model was built for a different t_max")
        if batch_loss not in ("sum", "mean"):
            raise ValueError("batch_loss must be 'sum' or 'mean'")
        self.shared_model = model          # device params are shared by construction
        self.model = model
        self.optimizer = optimizer
        if optimizer.target is None:
            optimizer.setup(model)
        self.t_max, self.gamma, self.beta = t_max, gamma, beta
        self.process_idx, self.clip_reward = process_idx, clip_reward
        self.phi = phi
        self.pi_loss_coef, self.v_loss_coef = pi_loss_coef, v_loss_coef
        self.keep_loss_scale_same = keep_loss_scale_same
        self.resize_mode = resize_mode
        self.pg = process_group
        self.world, self.rank = world_info(process_group)
        if model.frames in ("stacks", "states") and model.net.n_envs == 1:
            # a3c.py:73 feeds phi(state) to the model: uint8 screens for dqn_phi (bit-exact
            # scaling in the conv kernels), phi's f32 output for any other phi
            model.set_frames("stacks" if _is_dqn_phi(phi) else "states")
        model._bound = True
        self.net = model.net
        self.single = (self.net.stack or self.net.states) and self.net.n_envs == 1
        self.collectives = self.world > 1 if collectives is None else bool(collectives)
        if self.single and self.collectives:
            raise ValueError("A3C: the one-env act() drop-in updates at its own terminals, so ranks cannot "
                             "all-reduce in step; use an n-env model (act_batch / run_window) for data "
                             "parallelism, or collectives=False for independent learners per rank")
        if self.collectives and not dist_initialized():
            raise ValueError("A3C: collectives=True needs torch.distributed initialised")
        # the loss of the lockstep batch: the sum over envs (and ranks), or its mean
        scale = 1.0 if batch_loss == "sum" else 1.0 / (self.net.n_envs * (self.world if self.collectives else 1))
        self._vcoef = v_loss_coef * scale
        self.net.set_loss(pi_loss_coef * scale, keep_loss_scale_same)
        # no all-reduce between learn and update: the clip norm comes from the learner's conv reduce
        self.net.set_norm_fold(not self.collectives)
        self.t = 0          # env-steps taken (per env)
        self.t_start = 0    # a3c.py:56,152 (reference-contract act)
        self._episode_start = True
        self._copied = None
        self.net.reset()
        if self.single:
            dev = self.net.device
            pin = dev.type == "cuda"
            sdt = torch.float32 if self.net.states else torch.uint8
            self._h_stack = torch.empty((1, 4, 84, 84), dtype=sdt, pin_memory=pin)
            self._h_rd = torch.zeros(2, dtype=torch.float32, pin_memory=pin)
            self._d_stack = torch.empty((1, 4, 84, 84), dtype=sdt, device=dev)
            self._d_rd = torch.zeros(2, dtype=torch.float32, device=dev)
            self._d_done = torch.zeros(2, dtype=torch.uint8, device=dev)   # [0] = 0, [1] = 1
            self._d_done[1] = 1

    def sync_parameters(self):
        """a3c.py:63-65 -- a no-op: actors read the device parameters."""

    # ------------------------------------------------------------ window pieces
    def _overlap_allreduce(self) -> bool:
        """With > 1 rank (and a learner that runs in parts, i.e. not the
        Nature head) the gradient all-reduce is split in two: the FC / LSTM /
        heads section (all but ~12k of the parameters) starts as soon as the
        FC reduce is done and runs on the collective stream while the conv
        backward computes; only the conv section waits for it."""
        return self.collectives and OVERLAP_ALLREDUCE and self.net.arch != ARCH_FF_NATURE

    def _learn(self, stream=None):
        """The gradient part of the window; with the overlapped all-reduce it
        stops before the conv backward (finish_window runs that part)."""
        net = self.net
        if self._overlap_allreduce():
            net.learn_parts(range(LEARN_CONV), self.gamma, self.beta, self._vcoef, self.clip_reward,
                            stream=stream)
        else:
            net.learn(self.gamma, self.beta, self._vcoef, self.clip_reward, stream=stream)

    def _reduce_and_step(self, stream=None, conv=None):
        net = self.net
        main = stream if stream is not None else torch.cuda.current_stream(net.device)
        with torch.cuda.stream(main):          # the collectives order against `main`
            if self._overlap_allreduce():
                o = net.layout["0/2/W"][0]      # conv1 / conv2 live in [0, o)
                work = allreduce_grads(net.grads[o:], self.pg, async_op=True, force=True)
                if conv is not None:
                    conv()                      # e.g. a captured graph of the conv part
                else:
                    net.learn_parts([LEARN_CONV], self.gamma, self.beta, self._vcoef, self.clip_reward,
                                    stream=main)
                if work is not None:
                    work.wait()
                net.stamp(stream=main)          # (window timeline: the FC / heads section's wait)
                allreduce_grads(net.grads[:o], self.pg, force=True)
                net.stamp(stream=main)          # (the conv section)
            elif self.collectives:
                allreduce_grads(net.grads, self.pg, force=True)
                net.stamp(stream=main)
            self.optimizer.update(stream=main, advance_window=True)

    def _update(self, stream=None):
        self._learn(stream)
        self._reduce_and_step(stream)

    # ------------------------------------------------------------ reference-contract act
    def act(self, state, reward=None, is_state_terminal=None):
        """a3c.py:67-167.  One-env model: state = ALE.state (or what `phi`
        maps to dqn_phi's image of it), reward, is_state_terminal -> the
        sampled action (int), or None for a terminal state.  n-env models:
        act_batch."""
        if not self.single:
            return self.act_batch(state, reward, is_state_terminal)
        net, T = self.net, self.t_max
        terminal = bool(is_state_terminal)
        r = 0.0 if reward is None else float(np.clip(reward, -1, 1) if self.clip_reward else reward)
        if self._copied is not None:
            self._copied.synchronize()                  # the pinned buffers' last upload has landed
        self._h_rd[0] = r
        if not terminal:
            self._h_stack[0].numpy()[...] = self._phi_input(state)
            self._d_stack.copy_(self._h_stack, non_blocking=True)
        self._d_rd.copy_(self._h_rd, non_blocking=True)
        if net.device.type == "cuda":
            self._copied = torch.cuda.Event()
            self._copied.record()
        rew = self._d_rd[:1]
        L = self.t - self.t_start
        update = (terminal and self.t_start < self.t) or L == T          # a3c.py:77-78
        if update:
            if terminal:                                # R = 0 over the L steps since the last update
                net.observe_stack(L, None, rew, self._d_done[1:])
                net.truncate_window(L)
            else:                                       # bootstrap v(s) at the pre-update params (a3c.py:85)
                net.observe_stack(T, self._d_stack, rew, self._d_done[:1])
                net.act(T, mode=0)
            self._update()                              # a3c.py:88-144; the window advances (slot T -> 0)
            self.t_start = self.t                       # a3c.py:152
        if terminal:                                    # a3c.py:165-167
            self._episode_start = True
            return None
        slot = 0 if update else L
        if not update:
            net.observe_stack(slot, self._d_stack, rew, self._d_done[:1], force_reset=self._episode_start)
        self._episode_start = False
        net.act(slot, mode=1)                           # a3c.py:154-164, post-update params
        self.t += 1
        return int(net.step_outputs(slot)["actions"][0].item())

    def _phi_input(self, state) -> np.ndarray:
        """What the ring stores for phi(state) (a3c.py:73).  phi = dqn_phi
        (the device one): the 4 uint8 screens themselves (dqn_phi.py:12-13
        asserts) -- the conv kernels apply the /255.  Any other phi, or none
        (the identity, a3c.py:34): phi's output, which must be float32 (4,
        84, 84) (or (1, 4, 84, 84)) as Chainer's Convolution2D takes it."""
        if self.net.stack:
            x = np.asarray(state)
            if x.shape != (4, 84, 84) or x.dtype != np.uint8:
                raise ValueError("A3C.act: with phi=dqn_phi, state must be 4 uint8 84x84 screens (dqn_phi.py:12-13)")
            return x
        x = state if self.phi is None else self.phi(state)
        x = x.detach().cpu().numpy() if torch.is_tensor(x) else np.asarray(x)
        x = x.reshape(x.shape[-3:]) if x.ndim == 4 and x.shape[0] == 1 else x
        if x.shape != (4, 84, 84):
            raise ValueError(f"A3C.act: phi(state) has shape {x.shape}, need (4, 84, 84)")
        if x.dtype != np.float32:
            raise ValueError(f"A3C.act: phi(state) is {x.dtype}; the model takes float32 input "
                             "(use phi=asyncrl_amd.dqn_phi for uint8 ALE screens)")
        return x

    def act_batch(self, pairs: torch.Tensor, reward=None, is_state_terminal=None) -> torch.Tensor:
        """a3c.py:67-167, lockstep-batched.  pairs: (n, 2, 210, 160, 3) uint8
        device tensor (frame 4, frame 3 of the skip) -- for the Doom models
        the screens (n, H, W, 3), for frames="stacks" models the (n, 4, 84,
        84) stacks; reward: (n,) f32 (clipped to [-1, 1] as at a3c.py:69-70);
        is_state_terminal: (n,) uint8/bool, the transition into this
        observation ended the episode.  Returns the sampled actions (n,)
        int32 (a device copy)."""
        net, T = self.net, self.t_max
        r = None if reward is None else torch.as_tensor(reward, dtype=torch.float32, device=net.device).contiguous()
        d = None if is_state_terminal is None else \
            torch.as_tensor(is_state_terminal, device=net.device).to(torch.uint8).contiguous()
        pairs = pairs.contiguous()
        if self.t == 0:
            net.observe_act(0, pairs, r, d, 1, force_reset=True, resize_mode=self.resize_mode)
            ta = 0
        elif self.t % T == 0:
            net.observe_act(T, pairs, r, d, 1, resize_mode=self.resize_mode)   # bootstrap v(s_T), pre-update params
            self._update()
            net.act(0)                       # a3c.py:154-164 with post-update params
            ta = 0
        else:
            ta = self.t % T
            net.observe_act(ta, pairs, r, d, 1, resize_mode=self.resize_mode)
        self.t += 1
        return net.step_outputs(ta)["actions"].clone()

    def run_window(self, pair_pool, reward_pool, done_pool, pool_len: int, first: bool = False, stream=None,
                   split_update: bool = False, env_groups: int | None = None):
        """One full lockstep window over device-resident pools (graph
        capturable when first=False): T x (phi, forward, sample), bootstrap,
        learn, [all-reduce], clip + RMSProp, advance.

        env_groups=G > 1 splits the envs into G contiguous ranges whose T + 1
        forward steps run as independent chains on G streams (envs are
        independent until the learner sums their gradients); chain g starts
        one kernel after chain g - 1, so one chain's latency-bound kernels
        (policy, FC ticket reduce) overlap another's conv / phi.  The streams
        join before arl_learn.  Results are identical to env_groups=1.
        None picks DeviceNet.default_env_groups() (2 from 1,024 envs up: C3
        LSTM 1,024 envs 1.215 -> 1.162 ms at two chains of 512; at 512 envs one
        chain is faster since those launches run two envs a conv workgroup and
        64-row FC tiles, C4 0.497 vs 0.509-0.518 ms; profiles/r03/r3l)."""
        net, T = self.net, self.t_max
        groups = net.env_groups(net.default_env_groups() if env_groups is None else env_groups)
        if (WINDOW_C and len(groups) == 1 and not split_update and not self.collectives
                and net.arch == net.base_arch and net.base_arch in (ARCH_FF, ARCH_LSTM)):
            # one C call: T x (observe, act), bootstrap, learn, clip + RMSProp, advance (arl_run_window)
            net.run_window(pair_pool, reward_pool, done_pool, pool_len, first, self.resize_mode, self.gamma, self.beta,
                           self._vcoef, self.clip_reward, stream=stream, **self.optimizer.update_args())
            self.t += T
            return
        if len(groups) == 1:
            # FF: the learner's returns ride on the bootstrap policy launch (as arl_run_window does)
            fuse = FUSE_RETURNS and net.base_arch == ARCH_FF and net.arch != ARCH_FF_NATURE
            if fuse:
                net.set_returns_fusion(True, self.gamma, self.beta, self._vcoef, self.clip_reward)
            try:
                self._forward_chain(pair_pool, reward_pool, done_pool, pool_len, first, stream, None)
            finally:
                if fuse:
                    net.set_returns_fusion(False)
        else:
            main = stream if stream is not None else torch.cuda.current_stream(net.device)
            side = self._side_streams(len(groups) - 1)
            net.prepare(main)                        # stale FC planes rebuilt before the chains fork
            for s in side:
                s.wait_stream(main)                  # fork before any chain is issued
            chains = [self._chain_steps(pair_pool, reward_pool, done_pool, pool_len, first,
                                        main if g == 0 else side[g - 1], envs) for g, envs in enumerate(groups)]
            # the chains' launches are issued (captured) step-interleaved -- step t of chain 0, of chain 1,
            # ..., then step t + 1 -- so a graph replay hands every chain's first launches to the device early
            started = [None] * len(chains)
            live = list(range(len(chains)))
            step = 0
            while live:
                for g in list(live):
                    if step == 0 and g > 0 and started[g - 1] is not None:
                        side[g - 1].wait_event(started[g - 1])   # stagger: after chain g-1's first kernel
                    ev = next(chains[g], StopIteration)
                    if ev is StopIteration:
                        live.remove(g)
                    elif ev is not None:
                        started[g] = ev
                step += 1
            for s in side:
                main.wait_stream(s)
            stream = main
        self._learn(stream)
        if split_update:
            return
        self.finish_window(stream=stream)

    def _side_streams(self, k: int):
        have = getattr(self, "_side", [])
        while len(have) < k:
            have.append(torch.cuda.Stream(device=self.net.device))
        self._side = have
        return have[:k]

    def _forward_chain(self, pair_pool, reward_pool, done_pool, pool_len, first, stream, envs):
        """T x (observe, act) + the bootstrap observe / act for envs (all if
        None) on `stream`."""
        for _ in self._chain_steps(pair_pool, reward_pool, done_pool, pool_len, first, stream, envs):
            pass

    def _chain_steps(self, pair_pool, reward_pool, done_pool, pool_len, first, stream, envs):
        """_forward_chain as a generator that yields after each step's
        launches: for an env group, the first yield is an event recorded after
        the chain's first kernel (the first conv launch, with or without its
        observation), later ones None."""
        net, T = self.net, self.t_max
        ev = None
        stagger = envs is not None   # env groups: chain g starts after chain g-1's first kernel
        for t in range(T + 1):
            obs = t > 0 or first
            if stagger and ev is None:
                if obs:                                # the first kernel is the observation
                    net.observe(t, pair_pool, reward_pool, done_pool, pool_len, force_reset=(t == 0),
                                resize_mode=self.resize_mode, stream=stream, envs=envs)
                    ev = torch.cuda.Event()
                    ev.record(stream)
                    net.act(t, stream=stream, envs=envs)
                    yield ev
                    continue
                net.act(t, mode=1 | ACT_CONV_ONLY, stream=stream, envs=envs)
                ev = torch.cuda.Event()
                ev.record(stream)
                net.act(t, mode=1 | ACT_AFTER_CONV, stream=stream, envs=envs)
                yield ev
                continue
            if obs:
                net.observe_act(t, pair_pool, reward_pool, done_pool, pool_len, force_reset=(t == 0),
                                resize_mode=self.resize_mode, stream=stream, envs=envs)
            else:
                net.act(t, stream=stream, envs=envs)
            yield None

    def finish_window(self, stream=None, conv=None):
        """The rest of a window after run_window(split_update=True): [the conv
        backward when the all-reduce is overlapped -- `conv`, if given, runs
        it, e.g. conv_graph.replay], the gradient all-reduce, clip + RMSProp
        and the window advance."""
        self._reduce_and_step(stream, conv)
        self.t += self.t_max

    # ------------------------------------------------------------ checkpoints
    def save_model(self, model_filename: str):
        """a3c.py:181-185: the model and the optimizer state ('.opt') as
        Chainer-layout HDF5 files (serializers.save_hdf5)."""
        serializers.save_hdf5(model_filename, self.model)
        serializers.save_hdf5(model_filename + ".opt", self.optimizer)

    def load_model(self, model_filename: str):
        """a3c.py:169-179: load the model, and the optimizer state when
        '<file>.opt' exists (copy_param to a shared model is a no-op: the
        device parameters are shared)."""
        serializers.load_hdf5(model_filename, self.model)
        opt = model_filename + ".opt"
        if os.path.exists(opt):
            serializers.load_hdf5(opt, self.optimizer)
