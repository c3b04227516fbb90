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


def gather_records(rec: np.ndarray, dist, device="cpu", pair_index=None) -> np.ndarray:
    """All-gather per-rank record blocks of any size; returns (n_total, 18) ordered by global
    pair index.

    Ranks may hold different pair counts (i mod G with n_total % G != 0, or LPT shards), and a
    collective needs equal shapes, so every block is padded to the largest count. Each row
    carries its global pair index in an extra column (-1 on padding rows); the padding is
    dropped and the rows sorted by index after the gather. pair_index: the global index of each
    local row (default: rank-major, i.e. the counts of lower ranks + 0..P-1)."""
    import torch

    rec = np.ascontiguousarray(rec, dtype=np.float32).reshape(-1, RECORD_FLOATS)
    n = rec.shape[0]
    world, rank = dist.get_world_size(), dist.get_rank()
    cnt = torch.tensor([n], dtype=torch.int64, device=device)
    counts = [torch.zeros_like(cnt) for _ in range(world)]
    dist.all_gather(counts, cnt)
    counts = [int(c.item()) for c in counts]
    if pair_index is None:
        pair_index = sum(counts[:rank]) + np.arange(n)
    pair_index = np.asarray(pair_index, dtype=np.int64)
    if pair_index.shape != (n,):
        raise ValueError("one pair index per record")
    m = max(counts)
    buf = np.full((m, RECORD_FLOATS + 1), -1.0, np.float64)
    buf[:n, :RECORD_FLOATS] = rec
    buf[:n, RECORD_FLOATS] = pair_index
    t = torch.from_numpy(buf).to(device)
    out = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(out, t)
    allr = torch.cat(out, 0).cpu().numpy()
    allr = allr[allr[:, RECORD_FLOATS] >= 0]
    allr = allr[np.argsort(allr[:, RECORD_FLOATS], kind="stable")]
    return allr[:, :RECORD_FLOATS].astype(np.float32)


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
