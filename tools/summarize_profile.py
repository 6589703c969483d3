"""Summarize a tools/profile_round.sh run into profiles/<tag>/ (committed evidence):
kernel_stats.csv (rocprofv3 --stats), pmc_per_kernel.json and profiles/pmc_summary.json
(HBM bytes per launch = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024: the gfx950 FETCH_SIZE
under-count correction of MI355X_MICROARCH.md §HBM)."""
import csv, collections, json, shutil, sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
tag = sys.argv[1]
src = ROOT / "gpurun_out" / tag
dst = ROOT / "profiles" / tag
dst.mkdir(parents=True, exist_ok=True)
shutil.copy(src / "trace" / "run_kernel_stats.csv", dst / "kernel_stats.csv")
for f in ("trace.log",):
    lines = [l for l in (src / f).read_text().splitlines() if l.startswith("{")]
    if lines:
        (dst / "bench_line.json").write_text(lines[-1] + "\n")

def load(path, counter):
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            d[r["Kernel_Name"].split("(")[0].replace("void ", "")].append(float(r["Counter_Value"]))
    return d

f = load(src / "fetch" / "run_counter_collection.csv", "FETCH_SIZE")
w = load(src / "write" / "run_counter_collection.csv", "WRITE_SIZE")
per = {}
for k in sorted(set(f) | set(w)):
    fs = sum(f.get(k, [0])) / max(1, len(f.get(k, [])))
    ws = sum(w.get(k, [0])) / max(1, len(w.get(k, [])))
    per[k] = {"launches": len(f.get(k, [])), "FETCH_SIZE_KB": fs, "WRITE_SIZE_KB": ws,
              "hbm_bytes_per_launch": 2 * fs * 1024 + ws * 1024}
(dst / "pmc_per_kernel.json").write_text(json.dumps(per, indent=1) + "\n")
summary = {"source": f"profiles/{tag}/pmc_per_kernel.json (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes)",
           "kernels": {}}
for k, v in per.items():
    short = k.split("::")[-1].split("<")[0]
    summary["kernels"].setdefault(short, v)
(ROOT / "profiles" / "pmc_summary.json").write_text(json.dumps(summary, indent=1) + "\n")
print(open(dst / "kernel_stats.csv").read())
for k, v in per.items():
    print(f"{k:40s} {v['hbm_bytes_per_launch']/1e6:10.2f} MB/launch")
