"""RMSpropAsync + GradientClipping, mirroring rmsprop_async.py:7-38 and the
Chainer hook used at a3c_ale.py:224-226.

The reference's update is `ms = alpha*ms + (1-alpha)*g*g; p -= lr*g/sqrt(ms+eps)`
(eps OUTSIDE the sqrt) per parameter array, CPU or a dormant CuPy
ElementwiseKernel.  Here it is one fused HIP kernel over the flat parameter
buffer (plus a norm pass when a GradientClipping hook is installed), bitwise
equal to update_one_cpu's f32 arithmetic.
"""
from __future__ import annotations

import torch

from ._lib import check, lib, ptr, stream_handle
from .net import nets_aliasing


class GradientClipping:
    """chainer.optimizer.GradientClipping(threshold) (a3c_ale.py:226)."""

    name = "GradientClipping"

    def __init__(self, threshold: float):
        self.threshold = float(threshold)


class RMSpropAsync:
    """rmsprop_async.py:7-21.  `lr` may be reassigned between updates (the
    reference anneals it every step, a3c_ale.py:111-112); for graph-captured
    windows set `anneal_total_steps` and the lr is annealed on the device."""

    def __init__(self, lr: float = 0.01, alpha: float = 0.99, eps: float = 1e-8):
        self.lr = lr
        self.alpha = alpha
        self.eps = eps
        self.hooks = []
        self.target = None
        self.anneal_total_steps = 0   # 0 = use self.lr as given
        self.n_total_envs = 0         # envs over all ranks (global_t per window)
        self._scratch = None
        self.t = 0                    # Chainer Optimizer.t / epoch (serialized into '.opt')
        self.epoch = 0

    def setup(self, model):
        """Chainer Optimizer.setup: bind the model whose flat params/grads and
        `ms` state (rmsprop_async.py:19-21, zero-initialised) are updated."""
        self.target = model
        return self

    def add_hook(self, hook):
        self.hooks.append(hook)

    @property
    def clip_threshold(self) -> float:
        for h in self.hooks:
            if isinstance(h, GradientClipping):
                return h.threshold
        return 0.0

    def update_args(self) -> dict:
        """The arguments of one update (net.optimize's, without the stream),
        counting it (Chainer's Optimizer.t)."""
        if self.anneal_total_steps > 0 and self.n_total_envs <= 0:
            # global_t per window = (window start + t_max) * n_total_envs: with 0
            # envs it never moves and the anneal would silently keep lr fixed
            raise ValueError("anneal_total_steps > 0 needs n_total_envs > 0 (envs over all ranks)")
        self.t += 1
        return dict(lr0=self.lr, total_steps=self.anneal_total_steps, n_total=self.n_total_envs, alpha=self.alpha,
                    eps=self.eps, clip=self.clip_threshold)

    def update(self, stream=None, advance_window=False):
        """GradientClipping hook(s) then update_one for every parameter,
        on the bound model's device buffers (a3c.py:139).  advance_window:
        also end the lockstep window (arl_optimize_advance)."""
        self.target.net.optimize(stream=stream, advance=advance_window, **self.update_args())

    def update_arrays(self, param: torch.Tensor, ms: torch.Tensor, grad: torch.Tensor, stream=None):
        """update_one on explicit flat f32 device tensors (the drop-in for
        RMSpropAsync.update_one_cpu / update_one_gpu on one array)."""
        clip = self.clip_threshold
        if clip > 0 and self._scratch is None:
            self._scratch = torch.zeros(1024, dtype=torch.float64, device=param.device)
        check(lib.arl_rmsprop(ptr(param), ptr(ms), ptr(grad), param.numel(), self.lr, self.alpha, self.eps,
                              clip, ptr(self._scratch) if clip > 0 else None, stream_handle(stream)),
              "arl_rmsprop")
        # the kernel wrote `param` behind torch's back: a net whose params it aliases rebuilds its
        # derived FC planes before the next forward
        for net in nets_aliasing(param):
            net.params_changed()
