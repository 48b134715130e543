"""Monte-Carlo trial sharding across GPUs (one process per GPU, torch.distributed).

The reference averages per-trial NMSE/LLF over Monte-Carlo trials
("Proposed method/Proposed_method_NMSEvsTp.py":154-176; SNR/all_Detectors.py:362-395).
Trials are independent, so they shard with NO data-path collective: rank g of G
owns trials {i : i mod G == g} of every sweep point, runs them through one
batched sbce_em call per point, and the only exchange is ONE all-reduce of the
per-point accumulators [sum NMSE, trial count, sum LLF per iteration] at the
end of the sweep (RCCL over xGMI with backend "nccl"; gloo in the CPU tests).

Determinism: each rank sums its trials in ascending trial order; the all-reduce
then adds G partial sums (order fixed by the backend), so 1/2/4/8-GPU results
agree to a few ulp of the mean.
"""
import numpy as np


def shard(n_trials, world, rank):
    """Trial indices owned by `rank` (strided, so every rank sees every sweep region)."""
    if not (0 <= rank < world):
        raise ValueError("rank out of range")
    return np.arange(rank, n_trials, world, dtype=np.int64)


def collective_device(dist):
    """Device an all-reduce buffer must live on for the initialised process group:
    the current HIP device for RCCL ("nccl"), None (host memory) otherwise."""
    if str(dist.get_backend()).lower() == "nccl":
        import torch
        return torch.device("cuda", torch.cuda.current_device())
    return None


class Accumulators:
    """Per-sweep-point sums, packed into one float64 vector for a single all-reduce."""

    def __init__(self, n_points, n_iters=0, n_extra=0):
        self.n_points = n_points
        self.n_iters = n_iters
        self.n_extra = n_extra
        self.nmse = np.zeros(n_points)
        self.count = np.zeros(n_points)
        self.llf = np.zeros((n_points, n_iters))
        self.extra = np.zeros((n_points, n_extra))    # e.g. SER sums (sweeps.ser_vs_snr)

    def add(self, point, nmse_values, llf_values=None, extra_values=None):
        v = np.sort(np.asarray(nmse_values, dtype=float).reshape(-1))   # order-independent
        self.nmse[point] += float(np.sum(v))
        self.count[point] += v.size
        if llf_values is not None and self.n_iters:
            self.llf[point] += np.sum(np.asarray(llf_values, dtype=float).reshape(-1, self.n_iters),
                                      axis=0)
        if extra_values is not None and self.n_extra:
            e = np.asarray(extra_values, dtype=float).reshape(-1, self.n_extra)
            self.extra[point] += np.sort(e, axis=0).sum(axis=0)

    def pack(self):
        return np.concatenate([self.nmse, self.count, self.llf.reshape(-1), self.extra.reshape(-1)])

    def unpack(self, vec):
        P, I, E = self.n_points, self.n_iters, self.n_extra
        self.nmse = vec[:P].copy()
        self.count = vec[P:2 * P].copy()
        self.llf = vec[2 * P:2 * P + P * I].reshape(P, I).copy()
        self.extra = vec[2 * P + P * I:].reshape(P, E).copy()
        return self

    def allreduce(self, dist=None, device=None):
        """ONE all-reduce(sum) of every accumulator (no-op when not distributed).

        RCCL ("nccl" backend) reduces device tensors only, so with that backend and no
        explicit `device` the vector goes to the current HIP device (gloo: host)."""
        if dist is None or not dist.is_available() or not dist.is_initialized():
            return self
        import torch
        t = torch.from_numpy(self.pack())
        if device is None:
            device = collective_device(dist)
        if device is not None:
            t = t.to(device)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        return self.unpack(t.cpu().numpy())

    def mean_nmse(self):
        return self.nmse / np.maximum(self.count, 1)

    def mean_llf(self):
        return self.llf / np.maximum(self.count, 1)[:, None]

    def mean_extra(self):
        return self.extra / np.maximum(self.count, 1)[:, None]
