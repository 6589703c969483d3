"""Per-kernel HBM traffic of the bench command (tools/bench_profile.sh output) ->
<out>/pmc_per_kernel.json + <out>/kernel_stats_headline.csv / kernel_stats_configs.csv.

  python tools/bench_pmc.py <tag> <out dir>

FETCH_SIZE and WRITE_SIZE come from separate --pmc passes of `bench.py --no-cpu --no-configs`
(the headline's calls only); hbm_bytes_per_launch = (2 * FETCH_SIZE + WRITE_SIZE) KiB * 1024
(the gfx950 FETCH_SIZE correction of MI355X_MICROARCH.md); avg_us from the kernel trace of the
default bench command (its headline part, tools/bench_kernel_stats.py)."""
import collections
import csv
import glob
import json
import shutil
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def short(name: str) -> str:
    return name.replace("void ", "").replace("mhs::", "").replace("(anonymous namespace)::", "").split("(")[0]


def counter(d: Path, cname: str):
    vals = collections.defaultdict(list)
    for f in glob.glob(str(d / "**" / "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == cname:
                vals[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    return vals


def main():
    tag, out = sys.argv[1], Path(sys.argv[2])
    src = ROOT / "gpurun_out" / tag
    out.mkdir(parents=True, exist_ok=True)
    for f in ("kernel_stats_headline.csv", "kernel_stats_configs.csv"):
        if (src / "bench_trace" / f).exists():
            shutil.copy(src / "bench_trace" / f, out / f)
    avg = {}
    if (out / "kernel_stats_headline.csv").exists():
        for r in csv.DictReader(open(out / "kernel_stats_headline.csv")):
            avg[short(r["Name"])] = float(r["AverageNs"]) / 1e3
    fe = counter(src / "bench_FETCH_SIZE", "FETCH_SIZE")
    wr = counter(src / "bench_WRITE_SIZE", "WRITE_SIZE")
    per = {}
    for k in sorted(set(fe) | set(wr)):
        f = sum(fe.get(k, [0.0])) / max(1, len(fe.get(k, [])))
        w = sum(wr.get(k, [0.0])) / max(1, len(wr.get(k, [])))
        b = (2 * f + w) * 1024
        us = avg.get(k)
        per[k] = {"launches_traced": len(fe.get(k, [])), "avg_us": us, "FETCH_SIZE_KB": f, "WRITE_SIZE_KB": w,
                  "hbm_bytes_per_launch": b,
                  "hbm_GBps": round(b / (us * 1e-6) / 1e9, 1) if us else None,
                  "frac_of_8TBps": round(b / (us * 1e-6) / 8e12, 4) if us else None}
    (out / "pmc_per_kernel.json").write_text(json.dumps(per, indent=1) + "\n")
    for k, v in per.items():
        print(f"{k[:44]:44s} us {v['avg_us'] or 0:8.1f}  MB {v['hbm_bytes_per_launch'] / 1e6:9.2f}  GB/s {v['hbm_GBps']}")


if __name__ == "__main__":
    main()
