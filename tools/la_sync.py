"""Synchronised calls (MHS_OPT_SYNC=1, no timing struct): host wall time per call, median of
`reps` batches of 10 calls -- the launch-ahead numeric A/B outside the bench's pipelined
steps.  usage: MHS_LAUNCH_AHEAD=0|1 python tools/la_sync.py <matrix>... [--reps N]"""
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "mh-spgemm_amd")]
import numpy as np  # noqa: E402
import mhspgemm  # noqa: E402
from mhspgemm import synth  # noqa: E402

args = [a for a in sys.argv[1:] if not a.startswith("--")]
reps = int(sys.argv[sys.argv.index("--reps") + 1]) if "--reps" in sys.argv else 7
tool = mhspgemm.Tool(0)
for name in args:
    if name.isdigit():
        continue
    A, _ = synth.load_or_synth(name)
    A.H2D(0)
    for _ in range(3):
        mhspgemm.spgemm(tool, A, A, timing=False)[0].release()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        for _ in range(10):
            mhspgemm.spgemm(tool, A, A, timing=False)[0].release()
        ts.append((time.perf_counter() - t0) / 10 * 1e3)
    hits, misses = tool.launch_ahead_calls()
    print(json.dumps({"matrix": name, "ms": round(float(np.median(ts)), 4), "la": os.environ.get("MHS_LAUNCH_AHEAD", "1"),
                      "hits": hits, "misses": misses}), flush=True)
    A.release()
tool.close()
