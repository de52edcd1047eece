"""bench.py's rank launcher: `--gpus N` started without torch.distributed.run runs N
ranks, one fresh process each, and forwards rank 0's one JSON line; a WORLD_SIZE other than --gpus is
an error.  CPU only: the ranks run a stub body over gloo (bench.py stub_rank_body) in place of the
render, which needs a GPU.  The multi-GPU split it replaces is src/main.rs:194-211 (rayon workers)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR",
                                                            "MASTER_PORT", "LOCAL_WORLD_SIZE", "GROUP_RANK")}
    env.update({"OMP_NUM_THREADS": "1", "CUDA_VISIBLE_DEVICES": "", "HIP_VISIBLE_DEVICES": ""}, **kw)
    return env


def test_launcher_runs_n_ranks_and_forwards_one_line():
    p = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--stub-ranks"], capture_output=True, text=True,
                       timeout=240, env=_env(), cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, p.stdout
    out = json.loads(lines[0])
    assert out["stub"] and out["n_gpus"] == 2
    ranks = sorted(out["ranks"], key=lambda r: r["RANK"])
    assert [(r["RANK"], r["LOCAL_RANK"], r["WORLD_SIZE"]) for r in ranks] == [(0, 0, 2), (1, 1, 2)]
    assert len({r["pid"] for r in ranks}) == 2  # two fresh processes
    assert "torch.distributed.run" in p.stderr  # the launch it started, echoed


def test_world_size_mismatch_is_an_error():
    p = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--stub-ranks"], capture_output=True, text=True,
                       timeout=120, env=_env(RANK="0", LOCAL_RANK="0", WORLD_SIZE="1", MASTER_ADDR="127.0.0.1",
                                             MASTER_PORT="29999"), cwd=ROOT)
    assert p.returncode == 2
    assert "WORLD_SIZE 1" in p.stderr and not p.stdout.strip()


def test_too_few_gpus_fails_fast():
    """--gpus 2 where the node has fewer GPUs (none here) exits 2 with a clear message, no line."""
    p = subprocess.run([sys.executable, BENCH, "--gpus", "2"], capture_output=True, text=True, timeout=120,
                       env=_env(), cwd=ROOT)
    assert p.returncode == 2
    assert "needs 2 GPUs" in p.stderr and not p.stdout.strip()
