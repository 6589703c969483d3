"""Per-kernel statistics of the headline part of a `rocprofv3 --kernel-trace --stats -- python3 bench.py`
run: bench.py times the headline matrix first (warmup + steps pipelined calls, then 5 synchronised
phase calls and one cold call) and the configs block after it, so the rocprof --stats file mixes
the configs' launches of the same kernels into its averages.  This splits the kernel trace at the
first mask launch (k_mask_b / k_mask_lane) past the headline's calls and writes rocprof-style stats of each part.

  python tools/bench_kernel_stats.py <kernel_trace.csv> <out_dir> [warmup steps]
"""
import collections
import csv
import sys
from pathlib import Path


def main():
    trace, out = sys.argv[1], Path(sys.argv[2])
    warmup = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    steps = int(sys.argv[4]) if len(sys.argv) > 4 else 20
    rows = sorted(csv.DictReader(open(trace)), key=lambda r: int(r["Start_Timestamp"]))
    calls = warmup + steps + 5 + 1  # pipelined + phase calls + cold call
    seen, cut = 0, len(rows)
    for i, r in enumerate(rows):
        if "k_mask_" in r["Kernel_Name"]:  # k_mask_b or k_mask_lane
            seen += 1
            if seen == calls + 1:
                cut = i
                break
    out.mkdir(parents=True, exist_ok=True)
    for name, part in (("headline", rows[:cut]), ("configs", rows[cut:])):
        agg = collections.defaultdict(list)
        for r in part:
            agg[r["Kernel_Name"]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
        tot = sum(sum(v) for v in agg.values()) or 1
        with open(out / f"kernel_stats_{name}.csv", "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
            for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
                w.writerow([k, len(v), sum(v), round(sum(v) / len(v), 1), round(100.0 * sum(v) / tot, 2), min(v), max(v)])
        print(f"{name}: {len(part)} launches -> {out / f'kernel_stats_{name}.csv'}")


if __name__ == "__main__":
    main()
