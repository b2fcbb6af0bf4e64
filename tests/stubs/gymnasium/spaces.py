import numpy as np


class Box:
    """Test stub of gymnasium.spaces.Box (low / high / shape / dtype)."""

    def __init__(self, low, high, shape=None, dtype=np.float32, seed=None):
        self.dtype = np.dtype(dtype)
        low, high = np.asarray(low, self.dtype), np.asarray(high, self.dtype)
        self.shape = tuple(shape) if shape is not None else low.shape
        self.low = np.broadcast_to(low, self.shape).astype(self.dtype)
        self.high = np.broadcast_to(high, self.shape).astype(self.dtype)

    def contains(self, x):
        x = np.asarray(x)
        return bool(x.shape == self.shape and np.all(x >= self.low) and np.all(x <= self.high))
