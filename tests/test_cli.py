"""The `spgemm` CLI (mh-spgemm_amd/bin/spgemm): the reference driver surface
(src/main.cu:74-217) with its compile-time switches as flags -- AAT, the vendor
(rocSPARSE for cuSPARSE) row, CHECK_RESULT's "pass"/"error", WRITE's CSV lines."""
import subprocess
from pathlib import Path

import pytest

from _util import GOLDEN

ROOT = Path(__file__).resolve().parent.parent
CLI = ROOT / "mh-spgemm_amd" / "bin" / "spgemm"


def run(*args, timeout=120):
    return subprocess.run([str(CLI), *map(str, args)], capture_output=True, text=True, timeout=timeout)


def test_cli_usage_without_gpu():
    r = run()
    assert r.returncode == 255 and "Invalid Arguments." in r.stdout and "Usage:" in r.stdout
    r = run("--bogus", GOLDEN / "cage4_like_A.mtx")
    assert r.returncode == 255 and "Invalid Arguments." in r.stdout


@pytest.mark.gpu
def test_cli_square_vendor_check_csv(tmp_path):
    r = run("--iters", 2, "--warmup", 1, "--check", "--csv", tmp_path, GOLDEN / "cage4_like_A.mtx")
    assert r.returncode == 0, r.stdout + r.stderr
    out = r.stdout
    assert "SpGEMM Start!!!" in out and "SpGEMM   End!!!" in out
    assert "MH-SpGEMM runtime is" in out and "rocsparse:" in out
    assert "\npass\n" in out, out
    assert (tmp_path / "Gflops_MH-SpGEMM.csv").read_text().strip()
    assert (tmp_path / "Gflops_rocsparse.csv").read_text().strip()


@pytest.mark.gpu
def test_cli_nonsquare_rejected_and_aat(tmp_path):
    r = run(GOLDEN / "rect_AB_A.mtx")
    assert r.returncode == 0 and "C=AA must have rowA = colA. Exit." in r.stdout
    r = run("--aat", "--check", GOLDEN / "rect_AB_A.mtx")
    assert r.returncode == 0, r.stdout + r.stderr
    assert "\npass\n" in r.stdout, r.stdout
