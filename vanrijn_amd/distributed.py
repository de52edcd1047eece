"""Multi-GPU sharding of the path: samples split across ranks, one reduce of the records.

The path is embarrassingly parallel over (pixel, sample).  Rank r of N renders the whole tile for
sample indices [(step * N + r) * spp, +spp) -- the counter-based random stream
makes the union over ranks exactly the sample set of a one-GPU render of N * spp samples -- and
the merge-exact half of the per-pixel accumulation records ({sum X, Y, Z, weight}, contiguous:
vanrijn_amd/records.py) is summed onto rank 0 with one in-place collective (RCCL over xGMI on
MI355X, gloo on CPU in the tests).
Summing records merges disjoint sample sets the way AccumulationBuffer::merge_tile's weighted
blend does (accumulation_buffer.rs:62-85): mean = sum(colour_sum) / sum(weight).

`frame_step` is the one step both bench.py (RCCL, HIP renderer) and tests/test_distributed.py
(gloo, the oracle standing in for the renderer) run, so the CPU tests exercise bench.py's logic.
"""
import torch
import torch.distributed as dist

from . import records as R


def world_info(group=None):
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(group), dist.get_world_size(group)
    return 0, 1


def first_sample(step, rank, world, spp):
    """First sample index of `rank`'s shard in frame `step` (shards of `spp` samples per pixel)."""
    return (step * world + rank) * spp


def shard_spp(total_spp, world, split):
    """Samples per pixel one rank renders per frame: the whole `total_spp` (weak scaling, every GPU
    renders a full frame's worth) or `total_spp / world` (strong scaling: SURVEY.md 8(e)'s
    spp-split of one frame, C4 / C5)."""
    if not split:
        return total_spp
    if total_spp % world:
        raise ValueError(f"{total_spp} spp do not split evenly over {world} ranks")
    return total_spp // world


def reduce_bytes(state: torch.Tensor):
    """Bytes one rank contributes to the reduce: the 4 f64 sums of every pixel."""
    return R.sums(state).numel() * state.element_size()


def reduce_records(state: torch.Tensor, dst=0, group=None, timer=None, keep_local=False, via_host=False):
    """Sum per-rank accumulation records onto `dst` (in place; the one exchange of the path).

    Only the merge-exact sums {sum X, sum Y, sum Z, weight} travel -- 32 B per pixel, the records'
    first half, contiguous, reduced in place (no gather or scatter copies).  The Kahan
    compensations belong to no single update_pixel sequence once sums of different ranks are added
    (accumulation_buffer.rs:44-60), so `dst` zeroes them: an update_pixel continuation on the
    reduced state starts a fresh compensated sum from the merged totals.  On the other ranks the
    sums half belongs to the collective once called (in place: gloo uses it as scratch; the frame
    is done with it), their compensations are untouched.

    So after the call a rank other than `dst` holds NO valid records: its sums half is collective
    scratch, and an update_pixel continuation on it would silently build on garbage.  Callers that
    keep accumulating on every rank pass `keep_local=True`: the collective then runs on a copy of
    the sums half (32 B per pixel more HBM traffic), and the non-dst ranks' records stay their own.
    `timer`: a list that receives (start, end) CUDA events around everything this call enqueues (the
    collective and the zeroing).  `via_host`: the collective runs on a host copy of the sums half
    (a gloo group over device records: bench.py's one-GPU rehearsal of the N-rank path), the
    result copied back on `dst`."""
    rank, world = world_info(group)
    # through the collective whenever a group exists (at world size 1 too: bench.py under
    # torch.distributed.run on one GPU rehearses the RCCL step the 8-GPU runs take)
    if dist.is_available() and dist.is_initialized():
        flat = state.view(-1)
        sums = flat[:R.sums(flat).numel()]  # a contiguous view: the collective's buffer
        ev = None
        if timer is not None and state.is_cuda:
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            ev[0].record()
        buf = sums.clone() if keep_local and rank != dst else sums
        if via_host and buf.is_cuda:
            host = buf.cpu()
            dist.reduce(host, dst=dst, op=dist.ReduceOp.SUM, group=group)
            if rank == dst:
                buf.copy_(host)
        else:
            dist.reduce(buf, dst=dst, op=dist.ReduceOp.SUM, group=group)
        if rank == dst:
            R.compensations(flat).zero_()
        if ev is not None:
            ev[1].record()
            timer.append(ev)
    return state


def mean_colour(state: torch.Tensor):
    """Mean XYZ [pixels, 3] of records (accumulation_buffer.rs:59: sum * (1 / weight))."""
    s = R.sums(state)
    w = s[:, 3:4]
    return torch.where(w != 0, s[:, 0:3] * (1.0 / w), torch.zeros_like(s[:, 0:3]))


def frame_step(render_shard, state: torch.Tensor, step, spp, group=None, timer=None, keep_local=False,
               via_host=False):
    """One frame on this rank: render_shard(first_sample, state) renders (or enqueues) this rank's
    `spp` samples per pixel into `state` (fresh records), then the records are reduced onto rank 0.
    Afterwards only rank 0's `state` is valid (the other ranks' sums half was the collective's
    scratch) unless `keep_local` (reduce_records).  Returns what render_shard returned (launch stats
    on the GPU)."""
    rank, world = world_info(group)
    out = render_shard(first_sample(step, rank, world, spp), state)
    reduce_records(state, group=group, timer=timer, keep_local=keep_local, via_host=via_host)
    return out
