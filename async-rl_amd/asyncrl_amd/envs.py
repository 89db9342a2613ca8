"""Env-side adapter: emulator frames -> the hot path's frame-pair input
(SURVEY §8(f) item 4).

The reference wraps ALE in `ale.ALE` (ale.py:11-161): frame skip 4 with the
screen before the 4th act kept for the max-of-two, a life loss treated as
terminal, up to 30 no-op starts, the game reset on game over, and it runs the
whole phi pre-stage (max, luminance, resize, stack) on the CPU.  Here the
phi pre-stage is the GPU kernel, so the adapter stops at the raw frame pair:

  ALEFramePairs  one emulator, the reference's stepping semantics verbatim
                 (same ALE calls in the same order, so the same frames,
                 rewards, terminals and no-op counts), returning
                 (frame 4, frame 3) pairs instead of processed screens;
  VecALE         N of them stepped by host worker threads (the emulator
                 releases the GIL in act()) into pinned host buffers, copied
                 to the device asynchronously, in the (n, 2, 210, 160, 3)
                 uint8 / reward / terminal layout A3C.act takes.

Batched convention: a step whose action ends the episode returns
done = 1, the reward of that step, and the FIRST pair of the next episode
(the env re-initialises at once -- the reference's train loop does the same
one act() call later, a3c_ale.py:117-124).  Host-side code, not a kernel.
"""
from __future__ import annotations

from concurrent.futures import ThreadPoolExecutor

import numpy as np
import torch

SCREEN = (210, 160, 3)


class ALEFramePairs:
    """ale.ALE (ale.py:11-161) up to the raw frame pair.

    `ale` is an ale_python_interface.ALEInterface (ROM already loaded) or
    anything with its methods (act, getScreenRGB, lives, game_over,
    reset_game, getMinimalActionSet).  `nullop_rng` draws the no-op count
    with .randint(0, max_start_nullops + 1) -- numpy's global RNG by
    default, exactly like the reference."""

    def __init__(self, ale, frame_skip: int = 4, treat_life_lost_as_terminal: bool = True,
                 max_start_nullops: int = 30, nullop_rng=None):
        if frame_skip != 4:
            raise ValueError("the reference's receive_action is written for frame_skip = 4 (ale.py:118)")
        self.ale = ale
        self.treat_life_lost_as_terminal = treat_life_lost_as_terminal
        self.max_start_nullops = max_start_nullops
        self.rng = nullop_rng if nullop_rng is not None else np.random
        self.legal_actions = ale.getMinimalActionSet()
        self.pair = np.zeros((2,) + SCREEN, np.uint8)   # (current, previous raw screen)
        self.initialize()

    @classmethod
    def from_rom(cls, rom_filename: str, seed: int, **kw):
        """ale.py:21-49 setup (repeat_action_probability 0, no colour
        averaging, seeded) on a real ALE; needs ale_python_interface."""
        try:
            from ale_python_interface import ALEInterface
        except ImportError as e:
            raise ImportError("ale_python_interface is not installed; pass an emulator object instead") from e
        if not 0 <= seed < 2 ** 16:
            raise ValueError("ALE's random seed must be represented by unsigned int")
        ale = ALEInterface()
        ale.setInt(b"random_seed", seed)
        ale.setFloat(b"repeat_action_probability", 0.0)
        ale.setBool(b"color_averaging", False)
        ale.loadROM(str.encode(rom_filename))
        return cls(ale, **kw)

    @property
    def number_of_actions(self) -> int:
        return len(self.legal_actions)

    @property
    def is_terminal(self) -> bool:                       # ale.py:98-103
        if self.treat_life_lost_as_terminal:
            return self.lives_lost or self.ale.game_over()
        return self.ale.game_over()

    def initialize(self) -> np.ndarray:
        """ale.py:141-161: reset on game over, no-op starts; the first
        observation pairs the screen with itself (max of equal frames)."""
        if self.ale.game_over():
            self.ale.reset_game()
        if self.max_start_nullops > 0:
            for _ in range(self.rng.randint(0, self.max_start_nullops + 1)):
                self.ale.act(0)
        self.reward = 0
        scr = self.ale.getScreenRGB()
        self.pair[0] = scr
        self.pair[1] = scr
        self.lives_lost = False
        self.lives = self.ale.lives()
        return self.pair

    def receive_action(self, action: int):
        """ale.py:111-139: 4 frames, the raw screen before the 4th act kept;
        stops early on a terminal.  Returns the summed reward; on a
        non-terminal step self.pair = (screen after act 4, screen before)."""
        assert not self.is_terminal
        rewards = []
        last = None
        for i in range(4):
            if i == 3:
                last = self.ale.getScreenRGB()
            rewards.append(self.ale.act(self.legal_actions[action]))
            self.lives_lost = self.lives > self.ale.lives()
            self.lives = self.ale.lives()
            if self.is_terminal:
                break
        if not self.is_terminal:
            self.pair[0] = self.ale.getScreenRGB()
            self.pair[1] = last
        self.reward = sum(rewards)
        return self.reward

    def step(self, action: int):
        """One batched-convention step: (pair, reward, done)."""
        r = self.receive_action(action)
        done = self.is_terminal
        if done:
            self.initialize()
        return self.pair, r, done


class VecALE:
    """N emulators -> device tensors for A3C.act.

        env = VecALE([make_ale(i) for i in range(N)], device="cuda")
        pairs, r, d = env.reset()                  # (N,2,210,160,3) u8, (N,) f32, (N,) u8
        a = agent.act(pairs, r, d)
        pairs, r, d = env.step(a)

    Each env draws its no-op counts from its own RandomState(seed + i) (the
    global RNG would make the counts depend on thread timing)."""

    def __init__(self, ales, device=None, seed: int = 0, workers: int = 8, **kw):
        self.n = len(ales)
        self.envs = [ALEFramePairs(a, nullop_rng=np.random.RandomState(seed + i), **kw) for i, a in enumerate(ales)]
        self.device = torch.device(device if device is not None else "cuda")
        pin = self.device.type == "cuda"
        self.h_pairs = torch.empty((self.n, 2) + SCREEN, dtype=torch.uint8, pin_memory=pin)
        self.h_rewards = torch.zeros(self.n, dtype=torch.float32, pin_memory=pin)
        self.h_dones = torch.zeros(self.n, dtype=torch.uint8, pin_memory=pin)
        self.d_pairs = torch.empty((self.n, 2) + SCREEN, dtype=torch.uint8, device=self.device)
        self.d_rewards = torch.zeros(self.n, dtype=torch.float32, device=self.device)
        self.d_dones = torch.zeros(self.n, dtype=torch.uint8, device=self.device)
        self.pool = ThreadPoolExecutor(max_workers=max(1, min(workers, self.n)))
        self._copied = None        # event after the last host -> device copy
        self._chunks = [list(range(i, self.n, max(1, min(workers, self.n)))) for i in range(max(1, min(workers, self.n)))]

    @property
    def number_of_actions(self) -> int:
        return self.envs[0].number_of_actions

    def _upload(self, stream=None):
        with torch.cuda.stream(stream) if stream is not None and self.device.type == "cuda" else _null():
            self.d_pairs.copy_(self.h_pairs, non_blocking=True)
            self.d_rewards.copy_(self.h_rewards, non_blocking=True)
            self.d_dones.copy_(self.h_dones, non_blocking=True)
            if self.device.type == "cuda":
                self._copied = torch.cuda.Event()
                self._copied.record()
        return self.d_pairs, self.d_rewards, self.d_dones

    def _host_free(self):
        """The pinned buffers may be rewritten once the previous copy landed."""
        if self._copied is not None:
            self._copied.synchronize()

    def reset(self, stream=None):
        self._host_free()
        hp = self.h_pairs.numpy()
        for i, e in enumerate(self.envs):
            hp[i] = e.pair
        self.h_rewards.zero_()
        self.h_dones.zero_()
        return self._upload(stream)

    def step(self, actions, stream=None):
        acts = actions.cpu().numpy() if torch.is_tensor(actions) else np.asarray(actions)
        self._host_free()
        hp, hr, hd = self.h_pairs.numpy(), self.h_rewards.numpy(), self.h_dones.numpy()

        def run(idx):
            for i in idx:
                pair, r, d = self.envs[i].step(int(acts[i]))
                hp[i] = pair
                hr[i] = r
                hd[i] = d

        list(self.pool.map(run, self._chunks))
        return self._upload(stream)

    def close(self):
        self.pool.shutdown(wait=True)


class _null:
    def __enter__(self):
        return None

    def __exit__(self, *a):
        return False
