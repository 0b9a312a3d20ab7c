"""Deterministic fake local trainer for FL state-machine tests (no model compute)."""
import numpy as np


class FakeTrainer:
    def __init__(self, table, delta=1.0, n_samples=10):
        self.table = table
        self.flat = np.zeros(table.total, np.float32)
        self.delta = delta
        self.n_samples = n_samples
        self.rounds = []

    def set_weights(self, arrays):
        self.flat = self.table.from_list(arrays)

    def get_weights(self):
        return self.table.to_list(self.flat)

    def train_round(self, cr):
        self.rounds.append(cr)
        for e in self.table.entries:
            self.flat[e.offset:e.offset + e.size] += self.delta
        return {"loss": 0.0, "accuracy": 1.0}
