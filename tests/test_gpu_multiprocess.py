"""Two processes render HIP shards of one frame on one MI355X and reduce them.

The 8-GPU runs are the driver's; this is the same path at world size 2 on the one GPU a box has:
two freshly spawned processes each create the scene on cuda:0, render their shard of samples with
the HIP kernel through vanrijn_amd.distributed.frame_step -- the step bench.py runs -- and reduce
the 32-B sums of every pixel with gloo (host copies of the device records).  Rank 0's reduced
records must hold exactly the union's sample counts and its mean within 1e-12 of one process
rendering the union of samples (only the summation order differs), for both layouts: every rank a
full frame (weak scaling, c1-c3) and one frame's spp split over the ranks (c4 / c5).  Replaces the
rayon split of main.rs:194-211.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from vanrijn_amd import distributed as D
from vanrijn_amd import records as R

pytestmark = pytest.mark.gpu

H, W, SEED = 64, 80, 0x5EED0001


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _scene():
    from vanrijn_amd import scenes
    return scenes.main_scene(scenes.displaced_mesh(16, scenes._BUNNY_BUMPS, 0xB0BB1E, 8, 0.04,
                                                   (1.25, 1.05, 1.15), (-1.7, -0.8, 0.0)))


def _worker(rank, world, port, total_spp, split, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    from vanrijn_amd.render import Tile, render_tile_device
    ds = _scene().device_scene(0)
    spp = D.shard_spp(total_spp, world, split)
    dev = torch.zeros(H * W * 8, dtype=torch.float64, device="cuda")
    host = torch.zeros(H * W * 8, dtype=torch.float64)
    stream = torch.cuda.current_stream()

    def shard(first, st):  # the HIP renderer, then a host copy for gloo
        stats = render_tile_device(ds, Tile(0, W, 0, H), H, W, spp, SEED, first, dev.data_ptr(), stream.cuda_stream,
                                   timed=True)
        st.copy_(dev.cpu())
        return first, stats["kernel_ms"]

    first, _ = D.frame_step(shard, host, 1, spp)
    firsts = [None] * world
    dist.all_gather_object(firsts, first)
    if rank == 0:
        np.save(out_path, host.numpy())
        np.save(out_path + ".firsts.npy", np.array(firsts))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("split", [False, True])
def test_two_processes_reduce_like_one_render(tmp_path, split):
    from vanrijn_amd.render import Tile, render_tile_device
    world, total_spp = 2, 8
    spp = D.shard_spp(total_spp, world, split)
    out = str(tmp_path / "rank0.npy")
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, total_spp, split, out)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    reduced = np.load(out)
    firsts = sorted(int(f) for f in np.load(out + ".firsts.npy"))
    assert firsts == [(1 * world + r) * spp for r in range(world)]  # disjoint, contiguous shards
    # one process rendering the union of both shards' samples
    ds = _scene().device_scene(0)
    dev = torch.zeros(H * W * 8, dtype=torch.float64, device="cuda")
    render_tile_device(ds, Tile(0, W, 0, H), H, W, world * spp, SEED, firsts[0], dev.data_ptr(),
                       torch.cuda.current_stream().cuda_stream, timed=True)
    single = dev.cpu().numpy()
    fr, fs = R.fields(reduced), R.fields(single)
    assert np.array_equal(fr["weight"], fs["weight"])
    assert np.array_equal(fr["weight"], np.full(H * W, float(world * spp)))
    assert (R.compensations(reduced) == 0).all()
    mr = D.mean_colour(torch.from_numpy(reduced)).numpy()
    ms = D.mean_colour(torch.from_numpy(single)).numpy()
    assert np.abs(mr - ms).max() <= 1e-12 * max(1.0, float(np.abs(ms).max()))
    assert (fr["colour_sum"] != 0).any()
