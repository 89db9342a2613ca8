"""SoftmaxPolicyOutput (policy_output.py:32-61), backed by device buffers.

The reference computes probs / log_probs / entropy / sampled actions lazily
(cached_property) from the logits of one forward.  Here the policy kernel
computes all of them in the forward itself and this class exposes the same
attribute names as views of those device buffers.  The kernel draws one
action per row, either sampled (action_indices) or greedy
(most_probable_actions); the forward's mode decides which one is available.
"""
from __future__ import annotations

import torch


class SoftmaxPolicyOutput:
    def __init__(self, outputs: dict, greedy: bool = False):
        self._o = outputs
        self._greedy = greedy

    @property
    def logits(self) -> torch.Tensor:
        return self._o["logits"]

    @property
    def probs(self) -> torch.Tensor:            # policy_output.py:41-43
        return self._o["probs"]

    @property
    def log_probs(self) -> torch.Tensor:        # policy_output.py:45-47
        return self._o["log_probs"]

    @property
    def action_indices(self) -> torch.Tensor:   # policy_output.py:49-51 (int32, device)
        if self._greedy:
            raise RuntimeError("this output was computed in greedy mode: use most_probable_actions")
        return self._o["actions"]

    @property
    def most_probable_actions(self) -> torch.Tensor:   # policy_output.py:37-39 (int32, device)
        if not self._greedy:
            raise RuntimeError("this output was computed in sampling mode: run the forward with deterministic=True")
        return self._o["actions"]

    @property
    def sampled_actions_log_probs(self) -> torch.Tensor:   # policy_output.py:53-57
        if self._greedy:
            raise RuntimeError("this output was computed in greedy mode")
        return self._o["action_log_probs"]

    @property
    def entropy(self) -> torch.Tensor:          # policy_output.py:59-61
        return self._o["entropy"]


def fc_softmax_policy_and_v(h: torch.Tensor, W_pi: torch.Tensor, b_pi: torch.Tensor, W_v: torch.Tensor,
                            b_v: torch.Tensor, seed: int = 0, step=None, step_offset: int = 0,
                            env_offset: int = 0, mode: int = 1, stream=None):
    """FCSoftmaxPolicy + FCVFunction heads (policy.py:53-58, v_function.py:29-34)
    on h: (n, 256) f32, through the policy kernel (arl_policy).

    mode 1 samples with Philox(seed; env_offset + row, step[0] + step_offset)
    (step: int64 device tensor), mode 2 takes the first argmax, mode 0 draws
    nothing.  Returns (SoftmaxPolicyOutput, v)."""
    from ._lib import check, lib, ptr, stream_handle

    n, A = h.shape[0], W_pi.shape[0]
    dev = h.device
    f = dict(dtype=torch.float32, device=dev)
    o = {"logits": torch.empty(n, A, **f), "probs": torch.empty(n, A, **f), "log_probs": torch.empty(n, A, **f),
         "v": torch.empty(n, **f), "entropy": torch.empty(n, **f),
         "actions": torch.empty(n, dtype=torch.int32, device=dev), "action_log_probs": torch.empty(n, **f)}
    if mode == 1 and step is None:
        step = torch.zeros(1, dtype=torch.int64, device=dev)
    check(lib.arl_policy(ptr(h.contiguous()), n, ptr(W_pi.contiguous()), ptr(b_pi.contiguous()),
                         ptr(W_v.contiguous()), ptr(b_v.contiguous()), A, seed, ptr(step), step_offset, env_offset,
                         mode, ptr(o["logits"]), ptr(o["probs"]), ptr(o["log_probs"]), ptr(o["v"]),
                         ptr(o["entropy"]), ptr(o["actions"]) if mode else None,
                         ptr(o["action_log_probs"]) if mode else None, stream_handle(stream)), "arl_policy")
    return SoftmaxPolicyOutput(o, greedy=(mode == 2)), o["v"]
