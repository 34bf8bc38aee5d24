"""ORACLE TOOLING ONLY — gym 0.25.2 Discrete/Box surface (see __init__.py)."""
import numpy as np


class Discrete:
    def __init__(self, n, start=0):
        self.n = int(n)
        self.start = int(start)
        self.np_random = np.random.Generator(np.random.PCG64(np.random.SeedSequence(None)))

    def seed(self, seed=None):
        self.np_random = np.random.Generator(np.random.PCG64(np.random.SeedSequence(seed)))
        return [seed]

    def sample(self):
        return int(self.start + self.np_random.integers(self.n))


class Box:
    def __init__(self, low, high, shape=None, dtype=np.float32):
        self.low, self.high, self.shape, self.dtype = low, high, shape, dtype
