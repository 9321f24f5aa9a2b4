"""Index-range sharding of independent verification units.

No data-path collective: every shard is verified independently and verdicts
are written in place.  The same split is implemented natively for in-process
multi-GPU calls in csrc/coa_runtime.cpp (`shard`)."""


def shard_ranges(n, parts):
    """[lo, hi) ranges g*n/parts .. (g+1)*n/parts (empty shards dropped)."""
    out = []
    for g in range(parts):
        lo, hi = n * g // parts, n * (g + 1) // parts
        if hi > lo:
            out.append((g, lo, hi))
    return out


def rank_slice(rank, world, n_per_rank):
    """Weak scaling (bench.py): rank r owns the global index range
    [r * n_per_rank, (r + 1) * n_per_rank)."""
    return rank * n_per_rank, (rank + 1) * n_per_rank


def max_over_ranks(value, dist=None, device=None):
    """Max of a per-rank float over the process group (timing aggregation)."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return value
    import torch

    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
