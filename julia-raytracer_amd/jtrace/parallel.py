"""Multi-GPU sharding of the hot path: one process per GPU, samples split into
contiguous global ranges, one collective at the end.

Every (pixel, sample) is independent and the RNG is keyed by the *global* sample index, so
rank r traces samples [r*S/N, (r+1)*S/N) of every pixel on its own GPU with no data-path
communication. Each rank's accumulator is the running mean of its shard (src/trace.jl:631-648
restricted to the shard); the image is the sample-weighted sum of the shard means:

    image = sum_r n_r * mean_r / S

computed by one sum-reduce (RCCL over xGMI with backend "nccl"; gloo on CPU in the tests).
"""
from __future__ import annotations


def shard_range(total_samples: int, world: int, rank: int) -> tuple[int, int]:
    return rank * total_samples // world, (rank + 1) * total_samples // world


def reduce_running_means(tensor, n_local: int, n_total: int, dist, dst: int = 0):
    """Sum-reduce sample-weighted shard means onto `dst`; returns the combined mean on `dst`
    (the partial sum elsewhere). `tensor` is left untouched."""
    part = tensor * float(n_local)
    dist.reduce(part, dst=dst, op=dist.ReduceOp.SUM)
    if dist.get_rank() == dst:
        part /= float(n_total)
    return part


def all_reduce_running_means(tensor, n_local: int, n_total: int, dist):
    part = tensor * float(n_local)
    dist.all_reduce(part, op=dist.ReduceOp.SUM)
    part /= float(n_total)
    return part
