"""SoftmaxPolicyOutput (policy_output.py:32-61), backed by device buffers.

The reference computes probs / log_probs / entropy / sampled actions lazily
(cached_property) from the logits of one forward.  Here the policy kernel
computes all of them in the forward itself (one wave per env) and this class
exposes the same attribute names as views of those device buffers.
"""
from __future__ import annotations

import torch


class SoftmaxPolicyOutput:
    def __init__(self, outputs: dict):
        self._o = outputs

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
        return self._o["actions"]

    @property
    def sampled_actions_log_probs(self) -> torch.Tensor:   # policy_output.py:53-57
        return self._o["action_log_probs"]

    @property
    def entropy(self) -> torch.Tensor:          # policy_output.py:59-61
        return self._o["entropy"]
