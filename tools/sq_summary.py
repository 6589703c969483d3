"""Per-kernel SQ counters (tools/sq_passes.sh) averaged per launch -> <out>/sq_per_kernel.json.
usage: python tools/sq_summary.py <tag> <matrix> <out dir>"""
import collections
import csv
import glob
import json
import sys
from pathlib import Path

tag, m, out = sys.argv[1], sys.argv[2], Path(sys.argv[3])
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"gpurun_out/{tag}/{m}/pmc_*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].replace("void ", "").replace("mhs::", "").replace("(anonymous namespace)::", "").split("(")[0]
        vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
res = {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in vals.items()}
out.mkdir(parents=True, exist_ok=True)
(out / "sq_per_kernel.json").write_text(json.dumps(res, indent=1) + "\n")
for k, cs in res.items():
    if "k_num" in k or "k_sym_common" in k:
        v = cs.get("SQ_WAVE_CYCLES", 0) or 1
        print(f"{k[:40]:40s} waves {cs.get('SQ_WAVES', 0):9.0f} valu {cs.get('SQ_INSTS_VALU', 0):12.0f} "
              f"lds {cs.get('SQ_INSTS_LDS', 0):11.0f} wait_any {cs.get('SQ_WAIT_ANY', 0) / v:.2f} "
              f"active_any {cs.get('SQ_ACTIVE_INST_ANY', 0) / v:.2f} lds_conf {cs.get('SQ_LDS_BANK_CONFLICT', 0):.0f}")
