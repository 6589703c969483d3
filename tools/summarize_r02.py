"""Summarize a tools/prof_r02.sh (+ prof_sq.sh) run into profiles/<tag>/ (committed evidence).

Per matrix: kernel_stats.csv (rocprofv3 --stats of tools/sweep.py), pmc_per_kernel.json
(per launch: average duration from the trace, FETCH_SIZE / WRITE_SIZE from separate --pmc
passes, HBM bytes = 2*FETCH_SIZE + WRITE_SIZE -- the gfx950 FETCH_SIZE correction of
MI355X_MICROARCH.md §HBM -- and the achieved GB/s over the launch's own duration), the
sweep line; then profiles/pmc_summary.json keyed by matrix (read by bench.py) and, when the
SQ passes ran, sq_counters.json (per kernel, per launch).
usage: python tools/summarize_r02.py <tag> [head]"""
import collections
import csv
import json
import shutil
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
tag = sys.argv[1]
head = sys.argv[2] if len(sys.argv) > 2 else subprocess.run(
    ["git", "rev-parse", "--short", "HEAD"], capture_output=True, text=True, cwd=ROOT).stdout.strip()
src = ROOT / "gpurun_out" / tag
dst = ROOT / "profiles" / tag
dst.mkdir(parents=True, exist_ok=True)
PEAK = 8000.0


def kname(full: str) -> str:
    """'void mhs::k_num_wave<10240, true, false>(mhs::NumArgs)' -> 'k_num_wave<10240, true, false>'"""
    s = full.replace("void ", "")
    s = s.split("(")[0]
    return s.split("mhs::")[-1]


def first(path: Path, pattern: str):
    fs = sorted(path.rglob(pattern))
    return fs[0] if fs else None


def counters(path: Path):
    d = collections.defaultdict(lambda: collections.defaultdict(list))
    if path is None:
        return d
    for r in csv.DictReader(open(path)):
        d[kname(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return d


summary_path = ROOT / "profiles" / "pmc_summary.json"
try:
    summary = json.loads(summary_path.read_text())
    if "matrices" not in summary:
        summary = {}
except Exception:
    summary = {}
summary.setdefault("matrices", {})
summary["head"] = head
summary["note"] = ("per matrix: numeric + other kernels of one tools/sweep.py call; hbm_bytes_per_call = "
                   "2*FETCH_SIZE + WRITE_SIZE (gfx950 correction), separate --pmc passes")

for mdir in sorted(p for p in src.iterdir() if p.is_dir() and (p / "trace").exists()):
    m = mdir.name
    od = dst / m
    od.mkdir(exist_ok=True)
    stats = first(mdir / "trace", "*kernel_stats.csv")
    trace = first(mdir / "trace", "*kernel_trace.csv")
    if stats:
        shutil.copy(stats, od / "kernel_stats.csv")
    dur = collections.defaultdict(list)
    if trace:
        for r in csv.DictReader(open(trace)):
            dur[kname(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    sweep = [l for l in (mdir / "sweep.log").read_text().splitlines() if l.startswith("{")] \
        if (mdir / "sweep.log").exists() else []
    sw = json.loads(sweep[-1]) if sweep else {}
    if sw:
        (od / "sweep.json").write_text(json.dumps(sw) + "\n")
    f = counters(first(mdir / "fetch", "*counter_collection.csv"))
    w = counters(first(mdir / "write", "*counter_collection.csv"))
    calls = (sw.get("reps", 5) + 3) if sw else 8
    per = {}
    for k in sorted(set(dur) | set(f) | set(w)):
        fv = f.get(k, {}).get("FETCH_SIZE", [])
        wv = w.get(k, {}).get("WRITE_SIZE", [])
        fs = sum(fv) / len(fv) if fv else None
        ws = sum(wv) / len(wv) if wv else None
        avg_us = sum(dur[k]) / len(dur[k]) if dur.get(k) else None
        e = {"launches_traced": len(dur.get(k, [])), "avg_us": round(avg_us, 2) if avg_us else None,
             "FETCH_SIZE_KB": fs, "WRITE_SIZE_KB": ws}
        if fs is not None and ws is not None:
            b = 2 * fs * 1024 + ws * 1024
            e["hbm_bytes_per_launch"] = b
            if avg_us:
                e["hbm_GBps"] = round(b / (avg_us * 1e-6) / 1e9, 1)
                e["frac_of_8TBps"] = round(b / (avg_us * 1e-6) / 1e9 / PEAK, 4)
        per[k] = e
    # launches per call: numeric kernels launch once per call (a bin's kernel), so per call =
    # per launch; the figure below is per call of the whole product
    (od / "pmc_per_kernel.json").write_text(json.dumps(per, indent=1) + "\n")
    tot_b = sum(v.get("hbm_bytes_per_launch", 0) * (v["launches_traced"] / 8 if v["launches_traced"] else 1)
                for v in per.values())
    summary["matrices"][m] = {
        "source": f"profiles/{tag}/{m}/pmc_per_kernel.json",
        "kernels": {k: {"avg_us": v["avg_us"], "hbm_bytes_per_call": v.get("hbm_bytes_per_launch"),
                        "hbm_GBps": v.get("hbm_GBps")} for k, v in per.items() if not k.startswith("__amd")},
        "sweep": sw,
    }
    print(f"== {m}  e2e {sw.get('total_e2e')} ms  {sw.get('gflops_e2e')} GFLOPS  nnzC {sw.get('nnzC')}")
    for k, v in sorted(per.items(), key=lambda kv: -(kv[1]["avg_us"] or 0)):
        if k.startswith("__amd"):
            continue
        hb = v.get("hbm_bytes_per_launch")
        print(f"   {k:48s} {v['avg_us'] or 0:9.1f} us  {(hb or 0)/1e6:9.2f} MB  {v.get('hbm_GBps') or 0:8.1f} GB/s")

summary_path.write_text(json.dumps(summary, indent=1) + "\n")

# SQ passes (bench command on one matrix): per kernel, per launch
sq = {}
for p in sorted(src.glob("sq_*")):
    if not p.is_dir():
        continue
    c = counters(first(p, "*counter_collection.csv"))
    for k, cs in c.items():
        for cn, vals in cs.items():
            sq.setdefault(k, {})[cn] = sum(vals) / len(vals)
if sq:
    (dst / "sq_counters.json").write_text(json.dumps(sq, indent=1) + "\n")
    print("== SQ counters (per launch)")
    for k, cs in sorted(sq.items()):
        if k.startswith("__amd"):
            continue
        print(f"   {k}")
        for cn, v in sorted(cs.items()):
            print(f"      {cn:24s} {v:16.0f}")
