"""Resumable mini-batch order: epoch-shuffled batch indices with checkpointable state.

The reference trains once with L-BFGS on the whole set (`Logistic Regression.ipynb:34`) and
cannot resume (``warm_start=False``). The DP SGD trainers draw their mini-batches from this
schedule: every epoch is a fresh permutation of the rank-local batch indices, drawn from one
seeded generator (the same on every rank, so replicas stay in lock step). Its state - epoch,
cursor inside the epoch, and the generator state the current permutation was drawn from - goes
into the native checkpoint (``TrainState.epoch / data_cursor / rng_state``), so a resumed run
visits exactly the batches the uninterrupted run would have.
"""
from __future__ import annotations

from typing import Optional

import numpy as np
import torch


class BatchSchedule:
    def __init__(self, n_batches: int, seed: int = 0, shuffle: bool = True):
        self.nb = max(1, int(n_batches))
        self.shuffle = shuffle
        self.g = torch.Generator().manual_seed(int(seed))
        self.epoch = 0
        self.cursor = 0
        self._draw()

    def _draw(self) -> None:
        self._rng_epoch = self.g.get_state().clone()  # the state this epoch's order is drawn from
        self.order = (torch.randperm(self.nb, generator=self.g) if self.shuffle else torch.arange(self.nb)).tolist()

    def next(self) -> int:
        j = self.order[self.cursor]
        self.cursor += 1
        if self.cursor == self.nb:
            self.epoch += 1
            self.cursor = 0
            self._draw()
        return j

    # ---- checkpoint state
    def rng_state(self) -> np.ndarray:
        return self._rng_epoch.numpy().copy()

    def restore(self, epoch: int, cursor: int, rng_state: Optional[np.ndarray]) -> None:
        if rng_state is not None:
            self.g.set_state(torch.from_numpy(np.ascontiguousarray(rng_state, dtype=np.uint8)))
        self._draw()
        self.epoch = int(epoch)
        if not 0 <= int(cursor) < self.nb:
            raise ValueError(f"data cursor {cursor} outside [0, {self.nb})")
        self.cursor = int(cursor)
