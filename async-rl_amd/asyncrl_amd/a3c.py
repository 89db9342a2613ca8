"""A3C agent and models on the MI355X hot path (drop-in for a3c.py / a3c_ale.py).

Reference surfaces kept: `A3CModel` (a3c.py:15-24: pi_and_v, reset_state,
unchain_backward), `A3CFF` / `A3CLSTM` (a3c_ale.py:28-70), `A3C` (a3c.py:27-185:
__init__ arguments, act(state, reward, is_state_terminal), sync_parameters,
load_model / save_model).

What changes: the reference runs one env per process and updates
shared parameters Hogwild-style whenever that env finishes a t_max window or
an episode.  Here N envs step in lockstep on the GPU; every t_max steps one
update is made from the sum of all envs' window-segment gradients at fixed
parameters (a terminal inside a window closes that env's segment with R = 0,
exactly like a3c.py:82-83), all-reduced over ranks with RCCL when
torch.distributed is initialised, then clipped (40) and applied by
RMSpropAsync.  Hogwild races are gone; replicas stay bitwise identical.

`act` takes the raw frame pair of each env (frame 3 and frame 4 of the
4-frame skip, ale.py:118-119,134-135) -- the phi pre-stage runs on the GPU --
together with the reward and terminal flag of the transition into it.
Following batched-env convention, a terminal env's observation is already the
first frame of its next episode (auto-reset); the reference spends a separate
act(.., is_state_terminal=True) call on the terminal state instead.
"""
from __future__ import annotations

import os

import numpy as np
import torch

from ._lib import (ACT_AFTER_CONV, ACT_CONV_ONLY, ARCH_FF, ARCH_FF_NATURE, ARCH_LSTM, ARCH_RGB, LEARN_CONV,
                   RESIZE_SCALAR)
from .distributed import allreduce_grads, world_info
from .net import DeviceNet, init_like_torch
from . import serializers
from .policy_output import SoftmaxPolicyOutput

# env groups: chain g starts after chain g-1's first kernel (ARL_GROUP_STAGGER=0: together)
STAGGER = os.environ.get("ARL_GROUP_STAGGER", "1") != "0"
# > 1 rank: split the gradient all-reduce around the conv backward (ARL_OVERLAP_ALLREDUCE=0: one call)
OVERLAP_ALLREDUCE = os.environ.get("ARL_OVERLAP_ALLREDUCE", "1") != "0"


class A3CModel:
    """a3c.py:15-24."""

    arch = ARCH_FF

    def __init__(self, n_actions: int, n_envs: int = 1, t_max: int = 5, seed: int = 0, env_offset: int = 0,
                 init_seed: int | None = 0, device=None):
        self.n_actions = n_actions
        self.net = DeviceNet(self.arch, n_actions, n_envs, t_max, env_offset=env_offset, seed=seed,
                             device=device)
        if init_seed is not None:
            self.net.load_params(init_like_torch(self.arch, n_actions, np.random.default_rng(init_seed)))

    def pi_and_v(self, state: torch.Tensor, keep_same_state: bool = False, deterministic: bool = False):
        """state: (n, 4, 84, 84) f32 (dqn_phi output).  FF only; the LSTM
        model's recurrent forward runs inside A3C.act.  The policy output is
        computed eagerly: action_indices holds a Philox draw, or, with
        deterministic=True, most_probable_actions holds the first argmax
        (the two eval modes of a3c_ale.py:73-89)."""
        mode = 2 if deterministic else 1
        self.net.forward_states(state.contiguous(), mode=mode)
        o = self.net.step_outputs(self.net.t_max)
        n = state.shape[0]
        o = {k: v[:n] for k, v in o.items()}
        return SoftmaxPolicyOutput(o, greedy=deterministic), o["v"]

    def reset_state(self):
        pass

    def unchain_backward(self):
        pass

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

    def pi_and_v(self, state, keep_same_state=False):
        raise NotImplementedError("A3CLSTM forward runs inside A3C.act (recurrent state is on device)")


class DoomA3CFF(A3CModel):
    """train_a3c_doom.py:25-38 A3CFF: NIPSDQNHead(n_input_channels=3) on the
    RGB screen (phi = train_a3c_doom.py:21-23, no frame stack) ->
    FCSoftmaxPolicy + FCVFunction.  pi_and_v takes rgb_phi output
    (n, 3, 84, 84); A3C.act takes the raw (n, H, W, 3) screens."""
    arch = ARCH_FF | ARCH_RGB


class DoomA3CLSTM(A3CModel):
    """train_a3c_doom.py:41-63 A3CLSTM: the RGB NIPS head -> L.LSTM(256, 256)
    -> policy + value; recurrent forward inside A3C.act."""
    arch = ARCH_LSTM | ARCH_RGB

    def pi_and_v(self, state, keep_same_state=False):
        raise NotImplementedError("DoomA3CLSTM forward runs inside A3C.act (recurrent state is on device)")


class A3C:
    """a3c.py:27-185, lockstep-batched.  One `act` call = one env-step of all
    n_envs envs; every t_max calls it also performs the update."""

    def __init__(self, model: A3CModel, optimizer, t_max: int, gamma: float, beta: float = 1e-2,
                 process_idx: int = 0, clip_reward: bool = True, phi=None, pi_loss_coef: float = 1.0,
                 v_loss_coef: float = 0.5, keep_loss_scale_same: bool = False, resize_mode: int = RESIZE_SCALAR,
                 process_group=None):
        if pi_loss_coef != 1.0 or keep_loss_scale_same:
            raise NotImplementedError("pi_loss_coef != 1 / keep_loss_scale_same are not supported yet")
        if model.net.t_max != t_max:
            raise ValueError("model was built for a different t_max")
        self.shared_model = model          # device params are shared by construction
        self.model = model
        self.optimizer = optimizer
        if optimizer.target is None:
            optimizer.setup(model)
        self.t_max, self.gamma, self.beta = t_max, gamma, beta
        self.process_idx, self.clip_reward = process_idx, clip_reward
        self.v_loss_coef = v_loss_coef
        self.resize_mode = resize_mode
        self.pg = process_group
        self.world, self.rank = world_info(process_group)
        self.t = 0          # env-steps taken (per env)
        self.net = model.net
        self.net.reset()

    def sync_parameters(self):
        """a3c.py:63-65 -- a no-op: actors read the device parameters."""

    # ------------------------------------------------------------ window pieces
    def _overlap_allreduce(self) -> bool:
        """With > 1 rank (and a learner that runs in parts, i.e. not the
        Nature head) the gradient all-reduce is split in two: the FC / LSTM /
        heads section (all but ~12k of the parameters) starts as soon as the
        FC reduce is done and runs on the collective stream while the conv
        backward computes; only the conv section waits for it."""
        return self.world > 1 and OVERLAP_ALLREDUCE and self.net.arch != ARCH_FF_NATURE

    def _learn(self, stream=None):
        """The gradient part of the window; with the overlapped all-reduce it
        stops before the conv backward (finish_window runs that part)."""
        net = self.net
        if self._overlap_allreduce():
            net.learn_parts(range(LEARN_CONV), self.gamma, self.beta, self.v_loss_coef, self.clip_reward,
                            stream=stream)
        else:
            net.learn(self.gamma, self.beta, self.v_loss_coef, self.clip_reward, stream=stream)

    def _reduce_and_step(self, stream=None, conv=None):
        net = self.net
        main = stream if stream is not None else torch.cuda.current_stream(net.device)
        with torch.cuda.stream(main):          # the collectives order against `main`
            if self._overlap_allreduce():
                o = net.layout["0/2/W"][0]      # conv1 / conv2 live in [0, o)
                work = allreduce_grads(net.grads[o:], self.pg, async_op=True)
                if conv is not None:
                    conv()                      # e.g. a captured graph of the conv part
                else:
                    net.learn_parts([LEARN_CONV], self.gamma, self.beta, self.v_loss_coef, self.clip_reward,
                                    stream=main)
                if work is not None:
                    work.wait()
                allreduce_grads(net.grads[:o], self.pg)
            else:
                allreduce_grads(net.grads, self.pg)
            self.optimizer.update(stream=main, advance_window=True)

    def _update(self, stream=None):
        self._learn(stream)
        self._reduce_and_step(stream)

    def act(self, pairs: torch.Tensor, reward=None, is_state_terminal=None) -> torch.Tensor:
        """a3c.py:67-167, batched.  pairs: (n, 2, 210, 160, 3) uint8 device
        tensor (frame 4, frame 3 of the skip) -- for the Doom models the
        screens (n, H, W, 3) uint8 instead; reward: (n,) f32 (clipped to
        [-1, 1] as at a3c.py:69-70); is_state_terminal: (n,) uint8/bool, the
        transition into this observation ended the episode.  Returns the
        sampled actions (n,) int32 (device)."""
        net, T = self.net, self.t_max
        r = None if reward is None else torch.as_tensor(reward, dtype=torch.float32, device=net.device).contiguous()
        d = None if is_state_terminal is None else \
            torch.as_tensor(is_state_terminal, device=net.device).to(torch.uint8).contiguous()
        pairs = pairs.contiguous()
        if self.t == 0:
            net.observe(0, pairs, r, d, 1, force_reset=True, resize_mode=self.resize_mode)
            net.act(0)
            ta = 0
        elif self.t % T == 0:
            net.observe(T, pairs, r, d, 1, resize_mode=self.resize_mode)
            net.act(T)                       # bootstrap v(s_T), pre-update params
            self._update()
            net.act(0)                       # a3c.py:154-164 with post-update params
            ta = 0
        else:
            ta = self.t % T
            net.observe(ta, pairs, r, d, 1, resize_mode=self.resize_mode)
            net.act(ta)
        self.t += 1
        return net.step_outputs(ta)["actions"]

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
        None picks DeviceNet.default_env_groups() (2 from 512 envs up: C3 LSTM
        1024 envs 1.628 -> 1.542 ms, C4 FF 512 envs 0.683 -> 0.641 ms; at 256
        envs one chain is faster, 0.414 vs 0.431-0.448 ms)."""
        net, T = self.net, self.t_max
        groups = net.env_groups(net.default_env_groups() if env_groups is None else env_groups)
        if len(groups) == 1:
            self._forward_chain(pair_pool, reward_pool, done_pool, pool_len, first, stream, None)
        else:
            main = stream if stream is not None else torch.cuda.current_stream(net.device)
            side = self._side_streams(len(groups) - 1)
            for s in side:
                s.wait_stream(main)                  # fork before any chain is issued
            started = None
            for g, envs in enumerate(groups):
                s = main if g == 0 else side[g - 1]
                if started is not None:
                    s.wait_event(started)            # stagger: after chain g-1's first kernel
                started = self._forward_chain(pair_pool, reward_pool, done_pool, pool_len, first, s, envs)
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
        None) on `stream`.  For an env group, returns an event recorded after
        the chain's first kernel (the first observe, or the conv launch of
        step 0 when the window starts from the previous bootstrap obs)."""
        net, T = self.net, self.t_max
        ev = None
        for t in range(T + 1):
            if t > 0 or first:
                net.observe(t, pair_pool, reward_pool, done_pool, pool_len, force_reset=(t == 0),
                            resize_mode=self.resize_mode, stream=stream, envs=envs)
            if envs is not None and ev is None and STAGGER:
                if t == 0 and not first:
                    net.act(t, mode=1 | ACT_CONV_ONLY, stream=stream, envs=envs)
                    ev = torch.cuda.Event()
                    ev.record(stream)
                    net.act(t, mode=1 | ACT_AFTER_CONV, stream=stream, envs=envs)
                    continue
                ev = torch.cuda.Event()
                ev.record(stream)
            net.act(t, stream=stream, envs=envs)
        return ev

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
