"""bench.py's multi-GPU step through RCCL, rehearsed on one GPU.

The driver runs bench.py on 2/4/8 GPUs as `python -m torch.distributed.run --nproc-per-node N ...
bench.py --gpus N`.  Under torch.distributed.run bench.py creates the RCCL ("nccl") process group
even at world size 1, so this test takes that exact code path on one MI355X: RCCL init with
`device_id`, the barriers around the timed region, the records' `dist.reduce` inside every frame
(vanrijn_amd/distributed.py frame_step) and the max-over-ranks `all_reduce` of the elapsed time.
The rank processes are children of this one (never an exec of a GPU-initialised process).
"""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.gpu
@pytest.mark.parametrize("streams", [1, 2])
def test_bench_under_torchrun_world_one(streams):
    """streams 2: the N > 1 default (frames alternate over two streams and record buffers, each
    frame's reduce issued from its own stream); PMC passes of rank 0 on the first run only."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", "1", "--config", "c2", "--steps", "3", "--warmup", "1",
           "--no-cpu-baseline", "--no-drop-in", "--streams", str(streams)] + (["--no-pmc"] if streams == 2 else [])
    p = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 1 and out["steps"] == 3 and out["config"]["streams"] == streams
    # two streams: the frames one after another are timed too (each frame's own latency)
    assert ("sequential" in out) == (streams == 2)
    assert out["config"]["parallelism"] == "spp-split x1, RCCL reduce"
    assert out["value"] > 0 and out["ms_per_step"] > 0
    # one frame of C2 is 512 x 512 x 64 samples; value = samples / max-over-ranks time
    assert abs(out["value"] - 512 * 512 * 64 / (out["ms_per_step"] * 1e3)) < 1e-3 * out["value"] + 1e-3


@pytest.mark.gpu
def test_bench_two_ranks_on_one_gpu():
    """bench.py's N > 1 path end to end on the one-GPU box: `bench.py --gpus 2 --one-gpu-rehearsal`
    starts its own torch.distributed.run (the launcher), both ranks render on cuda:0 and reduce through
    gloo on host copies of the sums (RCCL cannot put two ranks on one GPU).  Everything else is the
    8-GPU run's code: c3 split 128 + 128 over the ranks, two streams, the weak-scaling and sequential
    regions, max-over-ranks timing, rank 0's PMC passes on its shard while rank 1 waits in the final
    barrier, one JSON line."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--one-gpu-rehearsal", "--config", "c3",
           "--width", "256", "--height", "256", "--steps", "3", "--warmup", "1"]
    p = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=280)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["scaling"] == "strong" and out["config"]["spp_per_gpu"] == 128
    assert out["config"]["streams"] == 2 and "rehearsal" in out
    assert out["weak_scaling"]["spp_per_gpu"] == 256 and out["sequential"]["streams"] == 1
    # value: both ranks' samples over the max-over-ranks time
    assert abs(out["value"] - 2 * 256 * 256 * 128 / (out["ms_per_step"] * 1e3)) < 1e-3 * out["value"] + 1e-3
    assert out["reduce"]["bytes_per_step_per_rank"] == 256 * 256 * 32
    assert "shard" in out["roofline"] and out["roofline"].get("frac") is not None  # rank 0's PMC passes ran
