"""Deterministic fake local trainer for FL state-machine tests (no model compute)."""
import numpy as np


class FakeTrainer:
    def __init__(self, table, delta=1.0, n_samples=10, sleep_s=0.0):
        self.table = table
        self.sleep_s = sleep_s
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
        if self.sleep_s:
            import time
            time.sleep(self.sleep_s)
        for e in self.table.entries:
            self.flat[e.offset:e.offset + e.size] += self.delta
        return {"loss": 0.0, "accuracy": 1.0}


class FakeFlatTrainer(FakeTrainer):
    """FakeTrainer whose model is reduced IN PLACE as one flat torch buffer - the contract of the HIP engine's
    ``LocalFit.fedavg_device`` (the RCCL data plane's device path), on CPU. ``fail_bucket`` = k > 0: the per-bucket
    hook raises at the k-th bucket, i.e. the reduction is lost part-way (the earlier buckets already reduced, the
    whole buffer already pre-scaled)."""

    def __init__(self, table, delta=1.0, n_samples=10, fail_bucket=-1):
        super().__init__(table, delta, n_samples)
        self.fail_bucket = fail_bucket
        self.uploads = []

    def fedavg_device(self, aggregator, n_local):
        import torch
        t = torch.from_numpy(self.flat)              # shares memory with self.flat
        seen = [0]

        def hook(sl):
            seen[0] += 1
            if seen[0] == self.fail_bucket:
                raise RuntimeError(f"injected: collective lost after bucket {seen[0] - 1}")

        aggregator.fedavg_device(t, n_local, on_bucket=hook)
        return True

    def get_weights(self):
        self.uploads.append(self.flat.copy())
        return super().get_weights()
