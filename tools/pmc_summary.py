"""Per-matrix, per-kernel HBM traffic of a tools/prof.sh run (modes serial + pmc) -> committed
evidence under profiles/<tag>/<matrix>/ and a rebuilt profiles/pmc_summary.json (one head).

  python tools/pmc_summary.py <tag> <head> [matrix ...]

For every kernel of one tools/sweep.py call (--reps 2 after 3 warm-ups: 5 calls a process):
  launches_per_call, avg_us (the one-stream kernel trace, MHS_NUM_STREAMS=1), FETCH_SIZE and
  WRITE_SIZE per launch (KiB, separate --pmc passes), hbm_bytes_per_call =
  (2 * FETCH_SIZE + WRITE_SIZE) * 1024 * launches_per_call (the gfx950 FETCH_SIZE correction of
  MI355X_MICROARCH.md §HBM), achieved HBM GB/s of the launch, TCC hit rate (TCC_HIT_sum /
  (TCC_HIT_sum + TCC_MISS_sum)), and its bin class (the north_star's per-bin-class figure)."""
import collections
import csv
import glob
import json
import shutil
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
CALLS = 5  # tools/sweep.py --reps 2: 3 warm-up + 2 timed calls

# kernel (demangled prefix) -> bin class (include/mhspgemm.h sym_bins / num_bins)
CLASSES = [
    ("k_mask_b", "front: Form_mask_matrix_B"),
    ("k_mask_lane", "front: Form_mask_matrix_B (a lane per row)"),
    ("k_analyze_lane", "front: row analysis (a lane per row)"),
    ("k_analyze", "front: row analysis (symbolic binning)"),
    ("k_probe_publish", "front: numeric-first probe"),
    ("k_bin_list", "front: symbolic bin lists"),
    ("k_sym_common", "symbolic: wave 5 KiB bin + tiny sort classes"),
    ("k_sym_rare", "symbolic: 10 KiB waves, 1024-thread and global bins, near groups"),
    ("k_sym_block", "symbolic: 256-thread block bin"),
    ("k_near", "symbolic: near row groups"),
    ("k_scan", "numeric binning: row_ptr scan + classification"),
    ("k_split_bins", "numeric binning: block bins split by LDS need"),
    ("k_num_wave_direct<5120", "numeric: wave 5 KiB direct"),
    ("k_num_wave_direct<10240", "numeric: wave 10 KiB direct"),
    ("k_num_wave_hash<5120", "numeric: wave 5 KiB hash"),
    ("k_num_wave_hash<10240", "numeric: wave 10 KiB hash"),
    ("k_num_wave<10240, true", "numeric: row groups (wave 10 KiB)"),
    ("k_num_block<256", "numeric: 256-thread block"),
    ("k_num_block<1024, false", "numeric: 1024-thread block (hub rows)"),
    ("k_num_block<1024, true", "numeric: global-memory tables"),
    ("k_tiny_num_small", "numeric: tiny sort classes (W <= 32)"),
    ("k_tiny_num<64", "numeric: tiny sort classes (64 lanes)"),
    ("k_tiny_copy_rows", "numeric: numeric-first slot copy"),
    ("k_copy_hash", "numeric: slot copy + 5 KiB hash wave rows (one launch)"),
]


def short(name: str) -> str:
    n = name.replace("void ", "").replace("mhs::", "").replace("(anonymous namespace)::", "")
    return n.split("(")[0]


def bin_class(k: str) -> str:
    for p, c in CLASSES:
        if k.startswith(p):
            return c
    return "other"


def counters(d: Path, name: str):
    vals = collections.defaultdict(list)
    for f in glob.glob(str(d / "**" / "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == name:
                vals[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    return vals


def stats(d: Path):
    out = {}
    for f in glob.glob(str(d / "**" / "*kernel_stats.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            out[short(r["Name"])] = {"calls": int(r["Calls"]), "avg_us": float(r["AverageNs"]) / 1e3}
        shutil.copy(f, d.parent / "kernel_stats_serial.csv")
    return out


def main():
    tag, head = sys.argv[1], sys.argv[2]
    src = ROOT / "gpurun_out" / tag
    mats = [m for m in sys.argv[3:] if m != "--fresh"] or sorted(p.name for p in src.iterdir() if (p / "pmc_1").exists())
    sf = ROOT / "profiles" / "pmc_summary.json"
    # merged into the committed summary (--fresh: start over); every matrix names its head
    summary = {"matrices": {}}
    if sf.exists() and "--fresh" not in sys.argv:
        summary = json.loads(sf.read_text())
    mats = [m for m in mats if m != "--fresh"]
    for m in mats:
        d = src / m
        dst = ROOT / "profiles" / tag / m
        dst.mkdir(parents=True, exist_ok=True)
        st = stats(d / "serial")
        if (d / "kernel_stats_serial.csv").exists():
            shutil.copy(d / "kernel_stats_serial.csv", dst / "kernel_stats_serial.csv")
        for t in ("timeline.txt", "timeline_serial.txt"):
            if (d / t).exists():
                shutil.copy(d / t, dst / t)
        fe = counters(d / "pmc_1", "FETCH_SIZE")
        wr = counters(d / "pmc_2", "WRITE_SIZE")
        hit = counters(d / "pmc_3", "TCC_HIT_sum")
        mis = counters(d / "pmc_3", "TCC_MISS_sum")
        per = {}
        for k in sorted(set(fe) | set(wr) | set(st)):
            n = len(fe.get(k, [])) or len(wr.get(k, []))
            fkb = sum(fe.get(k, [0.0])) / max(1, len(fe.get(k, [])))
            wkb = sum(wr.get(k, [0.0])) / max(1, len(wr.get(k, [])))
            lpc = n / CALLS if n else (st.get(k, {}).get("calls", 0) / 8)
            per_launch = (2 * fkb + wkb) * 1024 if k in fe and k in wr else None
            avg = st.get(k, {}).get("avg_us")
            h, ms = sum(hit.get(k, [])), sum(mis.get(k, []))
            per[k] = {
                "bin_class": bin_class(k), "launches_per_call": round(lpc, 2), "avg_us": avg,
                "FETCH_SIZE_KiB": round(fkb, 1), "WRITE_SIZE_KiB": round(wkb, 1),
                "hbm_bytes_per_launch": per_launch,
                "hbm_bytes_per_call": per_launch * lpc if per_launch is not None else None,
                "hbm_GBps": round(per_launch / (avg * 1e-6) / 1e9, 1) if per_launch and avg else None,
                "tcc_hit": round(h / (h + ms), 3) if h + ms > 0 else None,
            }
        (dst / "pmc_per_kernel.json").write_text(json.dumps(per, indent=1) + "\n")
        summary["matrices"][m] = {"source": f"profiles/{tag}/{m}/pmc_per_kernel.json", "head": head, "kernels": per}
        print(f"== {m}")
        for k, v in per.items():
            print(f"  {k[:40]:40s} {v['bin_class'][:36]:36s} us {v['avg_us'] or 0:9.1f} "
                  f"GB/s {v['hbm_GBps'] or 0:8.1f} hit {v['tcc_hit']}")
    heads = sorted({v.get("head", "?") for v in summary["matrices"].values()})
    summary["head"] = heads[0] if len(heads) == 1 else ",".join(heads)
    summary["note"] = ("per matrix: every kernel of one tools/sweep.py call on the matrix's head (numeric bins "
                       "on one stream for attribution); hbm_bytes_per_call = (2*FETCH_SIZE + WRITE_SIZE) * 1024 "
                       "per launch x launches per call (gfx950 correction), separate --pmc passes; "
                       "tcc_hit = TCC_HIT_sum / (TCC_HIT_sum + TCC_MISS_sum)")
    sf.write_text(json.dumps(summary, indent=1) + "\n")


if __name__ == "__main__":
    main()
