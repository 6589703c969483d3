"""bench.py's N-rank launch logic (CPU only): `python bench.py --gpus N` without a launcher
starts N ranks itself, and --gpus beyond the visible GPUs is an error."""
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402


def test_check_gpus_rejects_missing_devices():
    bench.check_gpus(1, "nccl", 1)
    bench.check_gpus(8, "nccl", 8)
    with pytest.raises(SystemExit):
        bench.check_gpus(2, "nccl", 1)
    with pytest.raises(SystemExit):
        bench.check_gpus(0, "nccl", 8)
    bench.check_gpus(4, "gloo", 1)  # a rehearsal: every rank on the one GPU


def test_spawn_ranks_sets_rank_env(tmp_path):
    out = tmp_path / "ranks"
    out.mkdir()
    child = ("import os, pathlib; e = os.environ; "
             f"pathlib.Path(r'{out}', e['RANK']).write_text("
             "' '.join([e['RANK'], e['LOCAL_RANK'], e['WORLD_SIZE'], e['MASTER_ADDR'], e['MASTER_PORT']]))")
    rc = bench.spawn_ranks([sys.executable, "-c", child], 3, poll_s=0.05)
    assert rc == 0
    got = sorted(p.read_text().split() for p in out.iterdir())
    assert [g[:3] for g in got] == [["0", "0", "3"], ["1", "1", "3"], ["2", "2", "3"]]
    assert {g[3] for g in got} == {"127.0.0.1"} and len({g[4] for g in got}) == 1


def test_spawn_ranks_fails_when_one_rank_fails():
    # rank 1 fails at once, rank 0 would hang forever: the launcher returns rank 1's code and
    # ends rank 0 instead of waiting
    child = "import os, sys, time; r = int(os.environ['RANK']); sys.exit(3) if r == 1 else time.sleep(600)"
    rc = bench.spawn_ranks([sys.executable, "-c", child], 2, poll_s=0.05)
    assert rc == 3


def test_bare_bench_refuses_more_gpus_than_visible():
    # no GPU in this container: --gpus 2 must fail loudly before touching the GPU
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["MHS_BENCH_BACKEND"] = "nccl"
    p = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--steps", "1"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode != 0
    assert "GPU(s) visible" in p.stderr
