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
