"""Pipelined steady-state steps of the product (exactly bench.py's time_steps) for a list of
matrices: ms per step, numeric ms (hipEvents on the launch stream), and -- with --reps R --
R interleaved repetitions (median) so that two libraries can be A/B'd in one process.

usage: python tools/pipe.py cant mac_econ_fwd500 ... [--steps 20] [--reps 3] [--lib DIR]
  --lib DIR: libmhspgemm.so of DIR instead of the package's (A/B: one process per library)
One JSON line per (matrix, library) on stdout; progress on stderr.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "mh-spgemm_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("matrices", nargs="+")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--lib", default="")
    ap.add_argument("--no-events", action="store_true", help="no numeric-phase hipEvents in the timed steps")
    args = ap.parse_args()
    args.no_events |= os.environ.get("MHS_PIPE_NO_EVENTS", "0") != "0"  # (A/B variants are env strings)
    if args.lib:  # (read by mhspgemm._lib at import)
        os.environ["MHS_LIB"] = str(Path(args.lib) / "libmhspgemm.so")
    import numpy as np
    import torch

    import mhspgemm
    from mhspgemm import _lib as L
    from mhspgemm import synth

    libs = [args.lib]
    t_start = time.time()
    tool = mhspgemm.Tool(0)
    tool.set_stream(torch.cuda.current_stream(0).cuda_stream)
    for m in args.matrices:
        A, src = synth.load_or_synth(m)
        flop = mhspgemm.flop_count_np(A.col, A.ptr)
        A.H2D(0)
        steps = args.steps if A.M < 1_000_000 else max(3, args.steps // 2)
        ms_l, nm_l = [], []
        for r in range(args.reps):
            tool.set_option(L.MHS_OPT_SYNC, 0)
            tool.set_option(L.MHS_OPT_NUMERIC_EVENTS, 0 if args.no_events else steps)
            for _ in range(args.warmup):
                C, _ = mhspgemm.spgemm(tool, A, A, timing=False)
                C.release()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(steps):
                C, _ = mhspgemm.spgemm(tool, A, A, timing=False)
                C.release()
            torch.cuda.synchronize()
            ms_l.append((time.perf_counter() - t0) / steps * 1e3)
            nm_l.append(0.0 if args.no_events else float(np.mean(tool.numeric_ms(steps))))
            tool.set_option(L.MHS_OPT_SYNC, 1)
            tool.set_option(L.MHS_OPT_NUMERIC_EVENTS, 0)
        ms = float(np.median(ms_l))
        out = {"matrix": m, "lib": libs[0] or "pkg", "rows": A.M, "flop": flop, "ms": round(ms, 4),
               "ms_all": [round(x, 4) for x in ms_l], "numeric_ms": round(float(np.median(nm_l)), 4),
               "gflops": round(2.0 * flop / (ms * 1e-3) / 1e9, 2)}
        print(json.dumps(out), flush=True)
        print(f"[pipe {time.time() - t_start:6.1f}s] {m}: {ms:.4f} ms", file=sys.stderr, flush=True)
        A.d_release_csr()
        tool.release()
    tool.close()


if __name__ == "__main__":
    main()
