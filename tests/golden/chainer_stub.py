"""A minimal, torch-float64-backed stand-in for the parts of Chainer 1.8.1 that
the reference's hot-path modules touch, so that `a3c.py`, `policy_output.py`,
`policy.py`, `v_function.py`, `dqn_head.py`, `init_like_torch.py`,
`rmsprop_async.py` and the model classes of `a3c_ale.py:28-70` run VERBATIM
from /root/reference at fixture-generation time (tests/golden/gen_golden.py).

Test infrastructure only: nothing here ships, and nothing on the GPU box
imports it.  Chainer itself is absent from the image, so its
primitives are restated here from Chainer 1.8.1's documented semantics:

  * parameters are float32 NumPy arrays with float32 `.grad` (as in Chainer);
    every forward casts them to float64 torch leaves, so activations and the
    backward run in float64 and each parameter gradient is rounded to f32
    once (the "truth" the HIP path is compared against at 1e-5);
  * Linear: y = x.reshape(n, -1) W^T + b; Convolution2D: cross-correlation,
    no padding; relu / softmax / log_softmax / select_item / sum / reshape;
  * L.LSTM: upward Linear(in, 4 out) + lateral Linear(out, 4 out, nobias)
    (lateral skipped while h is None), F.lstm with the gates interleaved per
    unit (reshape(n, out, 4) -> a, i, f, o), c = tanh(a) sig(i) + sig(f) c,
    h = sig(o) tanh(c);
  * Optimizer.setup / add_hook / update (hooks in insertion order, then
    update_one per parameter in namedparams order), GradientClipping
    (sqrt of the per-array f32 dots summed as Python floats; g *= rate if
    rate < 1), compute_grads_norm.

Python scalars combine with Variables as float64 here (Chainer would round
them to float32 first); the difference is far below the 1e-5 tolerance.
"""
from __future__ import annotations

import collections
import functools
import math
import sys
import types
import weakref

import numpy as np
import torch

F64 = torch.float64
_LIVE_PARAMS: "weakref.WeakSet[Parameter]" = weakref.WeakSet()


def _t(x):
    if isinstance(x, Variable):
        return x._t
    if isinstance(x, torch.Tensor):
        return x
    return torch.as_tensor(np.asarray(x), dtype=F64) if np.asarray(x).dtype.kind == "f" else \
        torch.as_tensor(np.asarray(x))


class Variable:
    """chainer.Variable over a float64 torch tensor (autograd graph)."""

    def __init__(self, data, volatile=False):
        if isinstance(data, torch.Tensor):
            self._t = data
        else:
            a = np.asarray(data)
            self._t = torch.as_tensor(a, dtype=F64) if a.dtype.kind == "f" else torch.as_tensor(a)

    @property
    def data(self):
        return self._t.detach().numpy()

    @property
    def shape(self):
        return tuple(self._t.shape)

    def __len__(self):
        return self._t.shape[0]

    def unchain_backward(self):
        self._t = self._t.detach()

    def backward(self):
        t = self._t
        t.backward(torch.ones_like(t))
        for p in list(_LIVE_PARAMS):
            p._harvest()

    # arithmetic (Python scalars and Variables)
    def __add__(self, o):
        return Variable(self._t + _t(o))

    __radd__ = __add__

    def __sub__(self, o):
        return Variable(self._t - _t(o))

    def __rsub__(self, o):
        return Variable(_t(o) - self._t)

    def __mul__(self, o):
        return Variable(self._t * _t(o))

    __rmul__ = __mul__

    def __truediv__(self, o):
        return Variable(self._t / _t(o))

    def __neg__(self):
        return Variable(-self._t)

    def __pow__(self, k):
        return Variable(self._t ** k)

    def __repr__(self):
        return f"variable({self.data!r})"


class Parameter(Variable):
    """A link parameter: float32 NumPy `data` / `grad` (Chainer layout); a
    float64 leaf is (re)built from `data` whenever `data` has changed."""

    def __init__(self, array):
        self.data_ = np.asarray(array, np.float32)
        self.grad = np.zeros_like(self.data_)
        self._leaf = None
        self._src = None

    @property
    def data(self):
        return self.data_

    @data.setter
    def data(self, v):
        self.data_ = v

    @property
    def _t(self):
        if self._leaf is None or not np.array_equal(self._src, self.data_):
            self._src = self.data_.copy()
            self._leaf = torch.from_numpy(self.data_.astype(np.float64)).requires_grad_(True)
            _LIVE_PARAMS.add(self)
        return self._leaf

    def _harvest(self):
        if self._leaf is not None and self._leaf.grad is not None:
            self.grad += self._leaf.grad.numpy().astype(np.float32)
            self._leaf.grad = None

    def zerograd(self):
        self.grad = np.zeros_like(self.data_)

    def __deepcopy__(self, memo):
        p = Parameter(self.data_.copy())
        p.grad = self.grad.copy()
        return p


# ---------------------------------------------------------------- links
class Link:
    def __init__(self, **params):
        self.__dict__.setdefault("_param_names", [])
        for name, shape in params.items():
            self.add_param(name, shape)

    def add_param(self, name, shape):
        self.__dict__.setdefault("_param_names", [])
        setattr(self, name, Parameter(np.zeros(shape, np.float32)))
        self._param_names.append(name)

    def _children_named(self):
        return []

    def namedparams(self):
        for n in getattr(self, "_param_names", []):
            yield "/" + n, getattr(self, n)
        for cname, child in self._children_named():
            for path, p in child.namedparams():
                yield "/" + cname + path, p

    def params(self):
        for _, p in self.namedparams():
            yield p

    def links(self, skipself=False):
        if not skipself:
            yield self
        for _, child in self._children_named():
            yield from child.links()

    def zerograds(self):
        for p in self.params():
            p.zerograd()


class Chain(Link):
    def __init__(self, **links):
        super().__init__()
        self.__dict__.setdefault("_children", [])
        for name, link in links.items():
            setattr(self, name, link)
            self._children.append(name)

    def _children_named(self):   # Chainer 1.8 visits a Chain's children in sorted name order
        return [(n, getattr(self, n)) for n in sorted(self.__dict__.get("_children", []))]


class ChainList(Link):
    def __init__(self, *links):
        super().__init__()
        self.__dict__["_list"] = list(links)

    def _children_named(self):
        return [(str(i), c) for i, c in enumerate(self.__dict__.get("_list", []))]

    def __getitem__(self, i):
        return self._list[i]

    def __iter__(self):
        return iter(self._list)

    def __len__(self):
        return len(self._list)


class Linear(Link):
    def __init__(self, in_size, out_size, wscale=1, bias=0, nobias=False, initialW=None, initial_bias=None):
        super().__init__()
        self.add_param("W", (out_size, in_size))
        self.b = None
        if not nobias:
            self.add_param("b", (out_size,))
            self.b.data[...] = bias

    def __call__(self, x):
        xt = _t(x)
        y = xt.reshape(xt.shape[0], -1) @ self.W._t.T
        if self.b is not None:
            y = y + self.b._t
        return Variable(y)


class Convolution2D(Link):
    def __init__(self, in_channels, out_channels, ksize, stride=1, pad=0, wscale=1, bias=0, nobias=False,
                 use_cudnn=True, initialW=None, initial_bias=None):
        super().__init__()
        self.stride, self.pad = stride, pad
        self.add_param("W", (out_channels, in_channels, ksize, ksize))
        self.b = None
        if not nobias:
            self.add_param("b", (out_channels,))
            self.b.data[...] = bias

    def __call__(self, x):
        y = torch.nn.functional.conv2d(_t(x), self.W._t, None if self.b is None else self.b._t,
                                       stride=self.stride, padding=self.pad)
        return Variable(y)


def _lstm(c_prev, x):
    """F.lstm(c_prev, x) -> (c, h); gates interleaved per unit."""
    n, g = x.shape[0], x.shape[1]
    r = x.reshape(n, g // 4, 4)
    a, i, f, o = torch.tanh(r[:, :, 0]), torch.sigmoid(r[:, :, 1]), torch.sigmoid(r[:, :, 2]), \
        torch.sigmoid(r[:, :, 3])
    c = a * i + f * c_prev
    return c, o * torch.tanh(c)


class LSTM(Chain):
    def __init__(self, in_size, out_size):
        super().__init__(upward=Linear(in_size, 4 * out_size), lateral=Linear(out_size, 4 * out_size, nobias=True))
        self.state_size = out_size
        self.reset_state()

    def reset_state(self):
        self.h = None
        self.c = None

    def __call__(self, x):
        lstm_in = self.upward(x)._t
        if self.h is not None:
            lstm_in = lstm_in + self.lateral(self.h)._t
        c_prev = torch.zeros(lstm_in.shape[0], self.state_size, dtype=F64) if self.c is None else self.c._t
        c, h = _lstm(c_prev, lstm_in)
        self.c, self.h = Variable(c), Variable(h)
        return self.h


# ---------------------------------------------------------------- functions
def relu(x):
    return Variable(torch.relu(_t(x)))


def softmax(x):
    return Variable(torch.softmax(_t(x), dim=1))


def log_softmax(x):
    return Variable(torch.log_softmax(_t(x), dim=1))


def select_item(x, t):
    xt, idx = _t(x), _t(t).long()
    return Variable(xt[torch.arange(xt.shape[0]), idx])


def sum_(x, axis=None):
    xt = _t(x)
    return Variable(xt.sum() if axis is None else xt.sum(dim=axis))


def reshape(x, shape):
    return Variable(_t(x).reshape(tuple(shape)))


# ---------------------------------------------------------------- optimizer
def _sum_sqnorm(arrays):
    return sum(float(np.dot(a.ravel(), a.ravel())) for a in arrays)


class GradientClipping:
    name = "GradientClipping"

    def __init__(self, threshold):
        self.threshold = threshold

    def __call__(self, opt):
        norm = math.sqrt(_sum_sqnorm([p.grad for p in opt.target.params()]))
        rate = self.threshold / norm
        if rate < 1:
            for p in opt.target.params():
                p.grad *= rate


class Optimizer:
    def setup(self, link):
        self.target = link
        self.t = 0
        self.epoch = 0
        self._hooks = collections.OrderedDict()
        self._states = {}
        for name, p in link.namedparams():
            st = {}
            self.init_state(p, st)
            self._states[name] = st

    def init_state(self, param, state):
        pass

    def add_hook(self, hook, name=None):
        self._hooks[name or hook.name] = hook

    def compute_grads_norm(self):
        return math.sqrt(_sum_sqnorm([p.grad for p in self.target.params()]))


class GradientMethod(Optimizer):
    def update(self, lossfun=None, *args):
        for hook in self._hooks.values():
            hook(self)
        self.t += 1
        for name, p in self.target.namedparams():
            self.update_one(p, self._states[name])

    def update_one(self, param, state):
        self.update_one_cpu(param, state)


def install():
    """Register chainer, chainer.{functions,links,optimizer,cuda,serializers}
    and cached_property in sys.modules."""
    ch = types.ModuleType("chainer")
    fns = types.ModuleType("chainer.functions")
    lks = types.ModuleType("chainer.links")
    opt = types.ModuleType("chainer.optimizer")
    cuda = types.ModuleType("chainer.cuda")
    ser = types.ModuleType("chainer.serializers")
    ch.Variable, ch.Link, ch.Chain, ch.ChainList = Variable, Link, Chain, ChainList
    fns.relu, fns.softmax, fns.log_softmax = relu, softmax, log_softmax
    fns.select_item, fns.sum, fns.reshape = select_item, sum_, reshape
    lks.Linear, lks.Convolution2D, lks.LSTM = Linear, Convolution2D, LSTM
    opt.Optimizer, opt.GradientMethod, opt.GradientClipping = Optimizer, GradientMethod, GradientClipping
    cuda.get_array_module = lambda *a: np
    ch.functions, ch.links, ch.optimizer, ch.cuda, ch.serializers = fns, lks, opt, cuda, ser
    for name, m in (("chainer", ch), ("chainer.functions", fns), ("chainer.links", lks),
                    ("chainer.optimizer", opt), ("chainer.cuda", cuda), ("chainer.serializers", ser)):
        sys.modules[name] = m
    cp = types.ModuleType("cached_property")
    cp.cached_property = functools.cached_property
    sys.modules["cached_property"] = cp
