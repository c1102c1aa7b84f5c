"""Cyclical step-size schedule — the host-side scalar feed of the fused step.

Same interface and values as the reference's CyclicalSGMCMC
(methods/cyclical.py:12-74), including its integer/float cycle-length split:
the lr uses L = K // M (int, :32) while should_sample / last_in_cycle /
get_cycle_number use L = K / M (float, :53, :64, :72).  When K % M != 0 the lr
restarts drift away from the cycle numbers and last_in_cycle never fires
(quirk Q3); that is reproduced, not fixed, so chains match the reference.
"""
from __future__ import annotations

import numpy as np


class CyclicalSGMCMC:
    """alpha(k) = base_lr * (1 + cos(pi * pos(k))) / 2, pos in [0, 1) per cycle."""

    def __init__(self, base_lr, nbr_of_cycles, epochs, proportion_exploration=0.5):
        self.base_lr = base_lr
        self.number_of_cycles = nbr_of_cycles
        self.epochs = epochs
        self.proportion_exploration = proportion_exploration
        self.current_epoch = 0
        self.sample_at_bottom = True

    @staticmethod
    def _iteration(epoch, batch, batches_per_epoch):
        return epoch * batches_per_epoch + batch + 1  # 1-based global iteration k

    def _float_cycle(self, batches_per_epoch):
        return self.epochs * batches_per_epoch / self.number_of_cycles

    def calculate_lr(self, epoch, batch, batches_per_epoch):
        total = self.epochs * batches_per_epoch
        length = total // self.number_of_cycles
        k = self._iteration(epoch, batch, batches_per_epoch)
        pos = ((k - 1) % length) / length
        # exploration and sampling stages share the cosine (cyclical.py:39-45)
        return self.base_lr * (1 + np.cos(pos * np.pi)) / 2

    def should_sample(self, epoch, batch, batches_per_epoch):
        if not self.sample_at_bottom:
            return True
        length = self._float_cycle(batches_per_epoch)
        k = self._iteration(epoch, batch, batches_per_epoch)
        return ((k - 1) % length) / length >= self.proportion_exploration

    def last_in_cycle(self, epoch, batch, batches_per_epoch):
        k = self._iteration(epoch, batch, batches_per_epoch)
        return (k % self._float_cycle(batches_per_epoch)) == 0

    def get_cycle_number(self, epoch, batch, batches_per_epoch):
        k = self._iteration(epoch, batch, batches_per_epoch)
        return int((k - 1) // self._float_cycle(batches_per_epoch)) + 1
