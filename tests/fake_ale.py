"""Test infrastructure shared by tests/golden/gen_golden.py and the env
adapter tests: seeded synthetic Atari-shaped frames and a stand-in for
ale_python_interface.ALEInterface (absent here) with a scripted episode."""
import numpy as np


def synth_frames(rng, n, kind):
    """Synthetic 210x160x3 uint8 frames: uniform, sparse palette
    blocks on black ("Breakout-shaped"), all-255, all-0."""
    if kind == "uniform":
        return rng.integers(0, 256, (n, 210, 160, 3), dtype=np.uint8)
    if kind == "white":
        return np.full((n, 210, 160, 3), 255, np.uint8)
    if kind == "black":
        return np.zeros((n, 210, 160, 3), np.uint8)
    if kind == "palette":
        pal = rng.integers(0, 256, (16, 3), dtype=np.uint8)
        out = np.zeros((n, 210, 160, 3), np.uint8)
        for i in range(n):
            for _ in range(40):
                y, x = rng.integers(0, 200), rng.integers(0, 150)
                h, w = rng.integers(2, 10), rng.integers(2, 12)
                out[i, y:y + h, x:x + w] = pal[rng.integers(0, 16)]
        return out
    raise ValueError(kind)


class FakeALE:
    """Stand-in for ale_python_interface.ALEInterface serving seeded frames.
    Episode: lives 3, a life lost at frame 22, game over at frame 41."""

    def __init__(self):
        self.rng = np.random.default_rng(11)
        self.frame = 0
        self.start = 0
        self._lives = 3
        self._over = False
        self.served = []

    def setInt(self, *a): pass
    def setFloat(self, *a): pass
    def setBool(self, *a): pass
    def setString(self, *a): pass
    def loadROM(self, *a): pass
    def getFrameNumber(self): return 0
    def getMinimalActionSet(self): return [0, 1, 3, 4]

    def getScreenRGB(self):
        f = synth_frames(np.random.default_rng(1000 + self.frame), 1, "palette")[0]
        if self.frame % 7 == 3:
            f[::2, ::3] = 255
        return f

    def act(self, a):
        self.frame += 1
        if self.frame - self.start == 22:
            self._lives -= 1
        if self.frame - self.start >= 41:
            self._over = True
        return int(self.frame % 5 == 0)

    def lives(self): return self._lives
    def game_over(self): return self._over

    def reset_game(self):
        self.start = self.frame
        self._over = False
        self._lives = 3


class FakeALEActions(FakeALE):
    """FakeALE whose rewards also depend on the action taken (so an adapter
    that forwards the wrong action is caught); logs every action."""

    def __init__(self):
        super().__init__()
        self.actions = []

    def act(self, a):
        self.actions.append(int(a))
        r = super().act(a)
        return r + (2 if a == 3 and self.frame % 3 == 0 else 0)
