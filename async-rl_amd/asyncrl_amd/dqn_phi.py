"""Frame preprocessing surfaces: dqn_phi.dqn_phi (dqn_phi.py:4-17), the
arithmetic of ale.ALE.current_screen (ale.py:59-89) + the 4-frame stack
(ale.py:135,155-158), and the ViZDoom phi (train_a3c_doom.py:21-23), batched
on the GPU.

All inputs are device tensors; the computation is libasyncrl_hip.so.
"""
from __future__ import annotations

import torch

from ._lib import RESIZE_SCALAR, check, lib, ptr, stream_handle


def _as_stack(screens) -> torch.Tensor:
    if isinstance(screens, (list, tuple)):
        assert len(screens) == 4
        screens = torch.stack([torch.as_tensor(s) for s in screens])
    return screens


def dqn_phi(screens, stream=None) -> torch.Tensor:
    """dqn_phi.py:4-17: 4 uint8 (84, 84) screens -> float32 (4, 84, 84) / 255.
    Also accepts a batch (n, 4, 84, 84) uint8 device tensor -> (n, 4, 84, 84)."""
    x = _as_stack(screens)
    single = x.dim() == 3
    if single:
        x = x.unsqueeze(0)
    assert x.dtype == torch.uint8 and tuple(x.shape[1:]) == (4, 84, 84), "dqn_phi: (n,4,84,84) uint8"
    x = x.to("cuda").contiguous()
    out = torch.empty(x.shape, dtype=torch.float32, device=x.device)
    check(lib.arl_dqn_phi(ptr(x), ptr(out), x.shape[0], stream_handle(stream)), "arl_dqn_phi")
    return out[0] if single else out


def current_screen(rgb_cur: torch.Tensor, rgb_prev: torch.Tensor, resize_mode: int = RESIZE_SCALAR,
                   stream=None) -> torch.Tensor:
    """ale.py:59-89 on (n, 210, 160, 3) uint8 device tensors -> (n, 84, 84)."""
    assert rgb_cur.shape == rgb_prev.shape and tuple(rgb_cur.shape[1:]) == (210, 160, 3)
    n = rgb_cur.shape[0]
    out = torch.empty((n, 84, 84), dtype=torch.uint8, device=rgb_cur.device)
    check(lib.arl_current_screen(ptr(rgb_cur), ptr(rgb_prev), ptr(out), n, resize_mode, stream_handle(stream)),
          "arl_current_screen")
    return out


def max_luminance(rgb_cur: torch.Tensor, rgb_prev: torch.Tensor, stream=None) -> torch.Tensor:
    """ale.py:62-69: max of two (..., 3) uint8 RGB arrays -> float64
    luminance -> uint8 (..., )."""
    assert rgb_cur.shape == rgb_prev.shape and rgb_cur.shape[-1] == 3
    out = torch.empty(rgb_cur.shape[:-1], dtype=torch.uint8, device=rgb_cur.device)
    check(lib.arl_max_luminance(ptr(rgb_cur), ptr(rgb_prev), ptr(out), out.numel(), stream_handle(stream)),
          "arl_max_luminance")
    return out


def phi_stack(rgb_pairs: torch.Tensor, prev_stack: torch.Tensor, reset: torch.Tensor | None = None,
              out: torch.Tensor | None = None, resize_mode: int = RESIZE_SCALAR, stream=None) -> torch.Tensor:
    """Materialised stack update (ale.py:135 / :155-158), batched:
    rgb_pairs (n, 2, 210, 160, 3) -> out (n, 4, 84, 84)."""
    n = rgb_pairs.shape[0]
    assert tuple(rgb_pairs.shape[1:]) == (2, 210, 160, 3) and tuple(prev_stack.shape) == (n, 4, 84, 84)
    if out is None:
        out = torch.empty_like(prev_stack)
    check(lib.arl_phi_stack(ptr(rgb_pairs), ptr(prev_stack), ptr(reset), ptr(out), n, resize_mode,
                            stream_handle(stream)), "arl_phi_stack")
    return out


def rgb_phi(images: torch.Tensor, resize_mode: int = RESIZE_SCALAR, stream=None) -> torch.Tensor:
    """train_a3c_doom.py:21-23 phi, batched: (n, H, W, 3) uint8 RGB24 screens
    (doom_env.py:47; W % 16 == 0) -> cv2.resize to 84 x 84 per channel ->
    transpose(2, 0, 1) -> float32 / 255: (n, 3, 84, 84).  One screen
    (H, W, 3) -> (3, 84, 84)."""
    single = images.dim() == 3
    x = images.unsqueeze(0) if single else images
    assert x.dtype == torch.uint8 and x.dim() == 4 and x.shape[3] == 3, "rgb_phi: (n, H, W, 3) uint8"
    x = x.contiguous()
    n, H, W = x.shape[0], x.shape[1], x.shape[2]
    out = torch.empty((n, 3, 84, 84), dtype=torch.float32, device=x.device)
    check(lib.arl_rgb_phi(ptr(x), n, H, W, ptr(out), resize_mode, stream_handle(stream)), "arl_rgb_phi")
    return out[0] if single else out
