"""Multi-GPU plumbing for independent registration pairs.

Pairs are independent units: rank g registers its own shard with no data-path collective,
and the only exchange is one all-gather of the per-pair result records
{T float[16] column-major, iterations, inlier ratio} (72 B per pair) at the end of a step.
The collective runs on whatever backend the process group uses (RCCL over xGMI on MI355X,
gloo in the CPU tests).
"""
from __future__ import annotations

import numpy as np

RECORD_FLOATS = 18  # T[16], iterations, inlier ratio


def shard_pairs(n_pairs: int, world: int, rank: int, weights=None) -> list[int]:
    """Pair indices of `rank`. Without weights: i mod world == rank.
    With weights (e.g. N * log M per pair): longest-processing-time greedy, ties by index."""
    if world < 1 or not (0 <= rank < world):
        raise ValueError("rank out of range")
    if weights is None:
        return list(range(rank, n_pairs, world))
    w = np.asarray(weights, dtype=np.float64)
    if w.shape != (n_pairs,):
        raise ValueError("one weight per pair")
    load = np.zeros(world)
    owner = np.empty(n_pairs, dtype=np.int64)
    for i in sorted(range(n_pairs), key=lambda i: (-w[i], i)):
        g = int(np.argmin(load))
        owner[i] = g
        load[g] += w[i]
    return [i for i in range(n_pairs) if owner[i] == rank]


def pack_records(T: np.ndarray, iterations, inlier_ratio) -> np.ndarray:
    """(P, 18) float32 records from P column-major transforms and per-pair stats."""
    T = np.asarray(T, dtype=np.float32).reshape(-1, 16)
    rec = np.zeros((T.shape[0], RECORD_FLOATS), np.float32)
    rec[:, :16] = T
    rec[:, 16] = np.asarray(iterations, dtype=np.float32)
    rec[:, 17] = np.asarray(inlier_ratio, dtype=np.float32)
    return rec


def gather_records(rec: np.ndarray, dist, device="cpu") -> np.ndarray:
    """All-gather equally sized per-rank record blocks; returns (world * P, 18) in rank order."""
    import torch

    t = torch.from_numpy(np.ascontiguousarray(rec, dtype=np.float32)).to(device)
    world = dist.get_world_size()
    out = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(out, t)
    return torch.cat(out, 0).cpu().numpy()


def max_over_ranks(value: float, dist, device="cpu") -> float:
    import torch

    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t[0])


def sum_over_ranks(value: float, dist, device="cpu") -> float:
    import torch

    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t[0])
