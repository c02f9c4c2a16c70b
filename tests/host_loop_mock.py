"""A stand-in solver for the host loop tests (not a test module): lanes that need fixed iteration counts, the
lock-step iteration() of the serial / pipelined schedules and the straggler tail's tail_run(k0, k1), with the
statistics layout of solver.STAT_FIELDS ([0] = active lanes).  No device: it exercises solver.newton_loop /
tail_loop, the switch decision and its pairing of collectives across ranks."""
import numpy as np
import torch


class MockSolver:
    def __init__(self, need, tail_lanes=0, tail_chunk=16):
        self.need = np.asarray(need, dtype=np.int64)
        self.B = len(self.need)
        self.k = 0
        self.tail_lanes, self.tail_chunk = tail_lanes, tail_chunk
        self.n_iter = torch.zeros(self.B, dtype=torch.int32)
        self.events = []
        self.timeline = None

    def _stats(self):
        st = torch.zeros(8, dtype=torch.float64)
        st[0] = float((self.n_iter.numpy() < self.need).sum())
        return st

    def iteration(self):                      # every active lane runs iteration k
        act = self.n_iter.numpy() < self.need
        self.n_iter[torch.from_numpy(act)] += 1
        self.k += 1
        self.events.append(("it", self.k))
        return self._stats()

    def tail_run(self, k0, k1):               # every active lane runs its own iterations k0 .. k1-1
        assert k0 == self.k, (k0, self.k)
        n = self.n_iter.numpy().astype(np.int64)
        act = n < self.need
        assert (n[act] == k0).all()           # the lock-step state the tail starts from
        self.n_iter = torch.from_numpy(np.where(act, np.minimum(self.need, k1), n).astype(np.int32))
        self.k = k1
        self.events.append(("tail", k0, k1))
        return self._stats()

    def collect_timing(self):
        pass
