"""World-size-2 run of the multi-GPU sharding + reduce on CPU (gloo), with the oracle standing in
for the GPU renderer of each shard.  Checks the reduced image against one process rendering the
union of the sample sets."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from vanrijn_amd import distributed as D


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _small_scene():
    from vanrijn_amd import scenes
    return scenes.main_scene(scenes.displaced_mesh(10, scenes._BUNNY_BUMPS, 0xB0BB1E, 8, 0.04,
                                                   (1.25, 1.05, 1.15), (-1.7, -0.8, 0.0)))


def _records(buf):
    return np.concatenate([buf["colour_sum"], buf["colour_bias"], buf["weight"][..., None],
                           buf["weight_bias"][..., None]], axis=-1)


def _worker(rank, world, port, spp, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import oracle_ffi as O
    from vanrijn_amd.render import Tile
    orc = O.OracleScene(_small_scene().spec())
    tile = Tile(0, 24, 0, 20)

    def shard(first):
        buf = orc.render_tile(tile, 20, 24, spp, seed=17, first_sample=first, mode=O.MODE_PRUNED)
        return torch.from_numpy(_records(buf).copy())

    state = D.render_frame(shard, step=0, spp=spp)
    if rank == 0:
        np.save(out_path, state.numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_sharded_frame_matches_single_process(tmp_path):
    from oracle import oracle_ffi as O
    from vanrijn_amd.render import Tile
    spp, world = 3, 2
    out = str(tmp_path / "rank0.npy")
    mp.spawn(_worker, args=(world, _free_port(), spp, out), nprocs=world, join=True)
    reduced = np.load(out)
    orc = O.OracleScene(_small_scene().spec())
    single = _records(orc.render_tile(Tile(0, 24, 0, 20), 20, 24, world * spp, seed=17, mode=O.MODE_PRUNED))
    assert np.array_equal(reduced[..., 6], single[..., 6])  # weights: exact sample counts
    mean_r = D.mean_colour(torch.from_numpy(reduced)).numpy()
    mean_s = D.mean_colour(torch.from_numpy(single)).numpy()
    assert np.abs(mean_r - mean_s).max() < 1e-12


def test_first_sample_partition():
    seen = set()
    for step in range(3):
        for r in range(4):
            f = D.first_sample(step, r, 4, 8)
            block = set(range(f, f + 8))
            assert not (block & seen)
            seen |= block
    assert seen == set(range(3 * 4 * 8))
