"""World-size 2 and 4 runs of the multi-GPU step on CPU (gloo), with the oracle standing in for the
GPU renderer of each shard.

Every rank runs vanrijn_amd.distributed.frame_step -- the same function bench.py's step() calls
with the HIP renderer and RCCL -- for both layouts bench.py has: weak scaling (every rank renders
`spp` samples per pixel, c1-c3) and one frame's spp split over the ranks (c4 / c5).  The reduced
records on rank 0 must hold exactly the union's sample counts, its mean within 1e-12 of one
process rendering the union, and zeroed Kahan compensations (an update_pixel continuation then
starts a fresh compensated sum, accumulation_buffer.rs:44-60).
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

H, W, SEED = 20, 24, 17


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _small_scene():
    from vanrijn_amd import scenes
    return scenes.main_scene(scenes.displaced_mesh(10, scenes._BUNNY_BUMPS, 0xB0BB1E, 8, 0.04,
                                                   (1.25, 1.05, 1.15), (-1.7, -0.8, 0.0)))


def _records(buf):
    return R.from_fields(buf["colour_sum"], buf["colour_bias"], buf["weight"], buf["weight_bias"])


def _worker(rank, world, port, total_spp, split, steps, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import oracle_ffi as O
    from vanrijn_amd.render import Tile
    orc = O.OracleScene(_small_scene().spec())
    spp = D.shard_spp(total_spp, world, split)
    state = torch.zeros(H * W * 8, dtype=torch.float64)

    def shard(first, st):  # the oracle in place of render_tile_device (fresh records per frame)
        buf = orc.render_tile(Tile(0, W, 0, H), H, W, spp, seed=SEED, first_sample=first, mode=O.MODE_PRUNED)
        st.copy_(torch.from_numpy(_records(buf).reshape(-1)))
        return first

    firsts = [D.frame_step(shard, state, step, spp) for step in range(steps)]
    gathered = [None] * world
    dist.all_gather_object(gathered, firsts)
    if rank == 0:
        np.save(out_path, state.numpy())
        np.save(out_path + ".firsts.npy", np.array(gathered))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,split", [(2, False), (4, False), (2, True), (4, True)])
def test_sharded_frame_matches_single_process(tmp_path, world, split):
    from oracle import oracle_ffi as O
    from vanrijn_amd.render import Tile
    total_spp, steps = 4, 2
    spp = D.shard_spp(total_spp, world, split)
    out = str(tmp_path / "rank0.npy")
    mp.spawn(_worker, args=(world, _free_port(), total_spp, split, steps, out), nprocs=world, join=True)
    reduced = np.load(out)
    firsts = np.load(out + ".firsts.npy")
    # the last frame's shards are disjoint and contiguous: [(step*N + r)*spp, +spp)
    last = sorted(int(f[-1]) for f in firsts)
    assert last == [((steps - 1) * world + r) * spp for r in range(world)]
    union_first, union_spp = last[0], world * spp
    orc = O.OracleScene(_small_scene().spec())
    single = _records(orc.render_tile(Tile(0, W, 0, H), H, W, union_spp, seed=SEED, first_sample=union_first,
                                      mode=O.MODE_PRUNED))
    fr, fs = R.fields(reduced, (H, W)), R.fields(single, (H, W))
    assert np.array_equal(fr["weight"], fs["weight"])  # weights: exact sample counts
    assert (R.compensations(reduced) == 0).all()  # compensations zeroed on rank 0
    mean_r = D.mean_colour(torch.from_numpy(reduced)).numpy()
    mean_s = D.mean_colour(torch.from_numpy(single)).numpy()
    assert np.abs(mean_r - mean_s).max() < 1e-12
    # an update_pixel continuation on the reduced state == the same continuation of the union
    buf = dict(fr, colour=np.zeros((H, W, 3)))
    nxt = union_first + union_spp
    cont = orc.render_tile(Tile(0, W, 0, H), H, W, 2, seed=SEED, first_sample=nxt, mode=O.MODE_PRUNED,
                           accumulate=buf)
    both = orc.render_tile(Tile(0, W, 0, H), H, W, union_spp + 2, seed=SEED, first_sample=union_first,
                           mode=O.MODE_PRUNED)
    assert np.array_equal(cont["weight"], both["weight"])
    assert np.abs(cont["colour"] - both["colour"]).max() < 1e-12


def test_c3_frame_is_split_over_the_ranks(tmp_path):
    """bench.py's headline config (c3: one 1024^2 @256spp frame, 1/2/4/8 GPUs) is strong-scaled: at
    world size 2 each rank renders 128 of the frame's 256 spp, and rank 0's reduced records equal one
    process rendering all 256 -- exact weights, means within 1e-12 (src/main.rs:194-211's
    rayon split).  The frame is shrunk to H x W pixels for the oracle; the spp are c3's."""
    import importlib.util
    from oracle import oracle_ffi as O
    from vanrijn_amd.render import Tile
    spec = importlib.util.spec_from_file_location("bench", os.path.join(os.path.dirname(__file__), "..", "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    c3 = bench.CONFIGS["c3"]
    assert c3["split"] and c3["spp"] == 256 and (c3["width"], c3["height"]) == (1024, 1024)
    assert [D.shard_spp(c3["spp"], n, c3["split"]) for n in (1, 2, 4, 8)] == [256, 128, 64, 32]
    out = str(tmp_path / "rank0.npy")
    mp.spawn(_worker, args=(2, _free_port(), c3["spp"], c3["split"], 1, out), nprocs=2, join=True)
    reduced = np.load(out)
    firsts = sorted(int(f[-1]) for f in np.load(out + ".firsts.npy"))
    assert firsts == [0, 128]  # 128 + 128: the two halves of one frame's sample range
    orc = O.OracleScene(_small_scene().spec())
    single = _records(orc.render_tile(Tile(0, W, 0, H), H, W, 256, seed=SEED, first_sample=0, mode=O.MODE_PRUNED))
    fr, fs = R.fields(reduced, (H, W)), R.fields(single, (H, W))
    assert np.array_equal(fr["weight"], fs["weight"]) and float(fr["weight"].min()) == 256.0
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


def test_shard_spp():
    assert D.shard_spp(256, 8, False) == 256
    assert D.shard_spp(1024, 8, True) == 128 and D.shard_spp(256, 8, True) == 32
    with pytest.raises(ValueError):
        D.shard_spp(256, 3, True)


def test_reduce_is_a_no_op_on_one_process():
    s = torch.arange(16, dtype=torch.float64)
    assert torch.equal(D.reduce_records(s.clone()), s)  # no process group: nothing reduced or zeroed


def test_reduce_moves_only_the_sums():
    """32 B per pixel -- {sum X, sum Y, sum Z, weight} -- not the whole 64-B record,
    and they are the records' first half: one contiguous in-place buffer (no gather / scatter)."""
    state = torch.zeros(H * W * 8, dtype=torch.float64)
    assert D.reduce_bytes(state) == 32 * H * W
    s = R.sums(state)
    assert s.is_contiguous() and s.data_ptr() == state.data_ptr() and s.numel() == 4 * H * W
    assert R.compensations(state).data_ptr() == state.data_ptr() + 32 * H * W


def test_records_fields_round_trip():
    rng = np.random.default_rng(3)
    f = {"colour_sum": rng.normal(size=(H, W, 3)), "colour_bias": rng.normal(size=(H, W, 3)),
         "weight": rng.normal(size=(H, W)), "weight_bias": rng.normal(size=(H, W))}
    flat = R.from_fields(**f)
    assert flat.shape == (8 * H * W,)
    g = R.fields(flat, (H, W))
    assert all(np.array_equal(f[k], g[k]) for k in f)
    assert np.array_equal(R.sums(flat)[:, 3], f["weight"].reshape(-1))


def _keep_worker(rank, world, port, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rec = torch.arange(5 * 8, dtype=torch.float64) + 100 * rank
    mine = rec.clone()
    D.reduce_records(rec)
    if rank == 0:
        want = sum(torch.arange(5 * 8, dtype=torch.float64) + 100 * r for r in range(world))
        want[20:] = 0.0  # the compensations half
        assert torch.equal(rec, want)
    else:
        # the collective works in place: a non-destination rank's sums half is the collective's
        # (gloo uses it as scratch), its compensations are untouched
        assert torch.equal(rec[20:], mine[20:])
    # keep_local: the collective runs on a copy on the other ranks, whose records stay their own
    rec2 = torch.arange(5 * 8, dtype=torch.float64) + 100 * rank
    D.reduce_records(rec2, keep_local=True)
    if rank == 0:
        assert torch.equal(rec2, want)
    else:
        assert torch.equal(rec2, mine)
    np.save(f"{out_path}.{rank}.npy", rec.numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_reduce_destination_and_other_ranks(tmp_path):
    out = str(tmp_path / "keep")
    mp.spawn(_keep_worker, args=(3, _free_port(), out), nprocs=3, join=True)
    assert all(os.path.exists(f"{out}.{r}.npy") for r in range(3))


def test_accumulation_buffer_from_state_shapes():
    """from_state takes the flat ABI-7 records with width / height, or a [h][w][8] array of them; a
    size that does not fit raises instead of misreading."""
    from vanrijn_amd.render import AccumulationBuffer
    rng = np.random.default_rng(4)
    f = {"colour_sum": rng.uniform(1, 2, size=(H, W, 3)), "colour_bias": rng.normal(size=(H, W, 3)) * 1e-17,
         "weight": rng.integers(1, 9, size=(H, W)).astype(float), "weight_bias": np.zeros((H, W))}
    flat = R.from_fields(**f)
    a = AccumulationBuffer.from_state(flat, W, H)
    b = AccumulationBuffer.from_state(flat.reshape(H, W, 8))
    c = AccumulationBuffer.from_state(torch.from_numpy(flat), W, H)
    for x in (b, c):
        assert np.array_equal(a.colour_buffer, x.colour_buffer) and np.array_equal(a.weight_buffer, x.weight_buffer)
    assert np.array_equal(a.colour_sum_buffer, f["colour_sum"])
    for bad in ((flat, W + 1, H), (flat.reshape(H, W * 8), None, None), (flat[: 8 * H * W - 8], W, H)):
        try:
            AccumulationBuffer.from_state(*bad)
        except ValueError:
            pass
        else:
            raise AssertionError("a record array of the wrong size must raise")
