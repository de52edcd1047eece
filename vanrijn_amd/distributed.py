"""Multi-GPU sharding of the path: samples split across ranks, one reduce of the records.

The path is embarrassingly parallel over (pixel, sample).  Rank r of N renders the whole tile for
sample indices [(step * N + r) * spp, +spp) -- the counter-based random stream
makes the union over ranks exactly the sample set of a one-GPU render of N * spp samples -- and
the per-pixel accumulation records (8 f64: sum XYZ, Kahan bias XYZ, weight, weight bias) are
summed onto rank 0 with one collective (RCCL over xGMI on MI355X, gloo on CPU in the tests).
Summing records merges disjoint sample sets the way AccumulationBuffer::merge_tile's weighted
blend does (accumulation_buffer.rs:62-85): mean = sum(colour_sum) / sum(weight).
"""
import torch
import torch.distributed as dist

RECORD = 8  # f64 per pixel


def first_sample(step, rank, world, spp):
    """First sample index of `rank`'s shard in frame `step`."""
    return (step * world + rank) * spp


def reduce_records(state: torch.Tensor, dst=0, group=None):
    """Sum per-rank accumulation records onto `dst` (in place; the one exchange of the path)."""
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.reduce(state, dst=dst, op=dist.ReduceOp.SUM, group=group)
    return state


def mean_colour(state: torch.Tensor):
    """Mean XYZ [.., 3] of records [.., 8] (accumulation_buffer.rs:59: sum * (1 / weight))."""
    s = state.reshape(-1, RECORD)
    w = s[:, 6:7]
    return torch.where(w != 0, s[:, 0:3] * (1.0 / w), torch.zeros_like(s[:, 0:3]))


def render_frame(render_shard, step, spp, group=None):
    """Run one frame on this rank: render_shard(first_sample) -> records tensor, then reduce.

    `render_shard` enqueues (GPU) or computes (CPU) this rank's records for samples
    [first_sample, first_sample + spp)."""
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    state = render_shard(first_sample(step, rank, world, spp))
    return reduce_records(state, group=group)
