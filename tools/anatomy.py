"""Variants of a stand-in for kernel attribution (a round-5 diagnostic run): scircuit-like with and
without its 20 hub rows / hub columns.  usage: python tools/anatomy.py <variant> -> pipelined
steps of that matrix (tools/pipe.py's loop), for a rocprofv3 kernel trace."""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "mh-spgemm_amd")]
import numpy as np  # noqa: E402


def scircuit_variant(rows: bool, cols: bool, seed: int = 5):
    from mhspgemm import synth
    n = 170_998
    rng = np.random.default_rng(seed)
    base = synth.banded_random(n, 4.0, 200, far_frac=0.1, seed=seed)
    hubs = rng.choice(n, size=20, replace=False)
    r = [np.repeat(np.arange(n), np.diff(base.ptr))]
    c = [base.col.astype(np.int64)]
    for h in hubs:
        others = rng.choice(n, size=350, replace=False)
        if rows:
            r.append(np.full(350, h)); c.append(others)
        if cols:
            r.append(others); c.append(np.full(350, h))
    return synth._csr_from_coo(n, n, np.concatenate(r), np.concatenate(c), rng)


def main():
    import torch
    import mhspgemm
    from mhspgemm import _lib as L
    v = sys.argv[1]
    A = scircuit_variant("rows" in v or v == "both", "cols" in v or v == "both")
    A.H2D(0)
    tool = mhspgemm.Tool(0)
    tool.set_stream(torch.cuda.current_stream(0).cuda_stream)
    tool.set_option(L.MHS_OPT_SYNC, 0)
    for _ in range(3):
        C, _ = mhspgemm.spgemm(tool, A, A, timing=False)
        C.release()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        C, _ = mhspgemm.spgemm(tool, A, A, timing=False)
        C.release()
    torch.cuda.synchronize()
    print(f"{v}: nnzA {A.nnz} {(time.perf_counter() - t0) / 10 * 1e3:.4f} ms per step", flush=True)
    tool.close()


if __name__ == "__main__":
    main()
